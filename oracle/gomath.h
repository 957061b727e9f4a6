// ORACLE — test infrastructure only (never linked into the product).
//
// Restatement of Go 1.16 `math` pure-Go algorithms used on the scoring path:
//   math.Pow  (src/math/pow.go)   — called by ScoreFitBinPack/ScoreFitSpread
//                                    (nomad/structs/funcs.go:241,267)
//   math.Exp  (src/math/exp.go, fdlibm e_exp.c)   — preemptionScore (rank.go:843)
//   math.Log  (src/math/log.go, fdlibm e_log.c)
//   math.Frexp/Ldexp/Modf (bit manipulation, exact)
// Go's amd64 build replaces Exp/Log with assembly; those bits are not
// reproducible without a Go toolchain. Policy: oracle
// and device use this portable algorithm and must agree bit-for-bit; parity
// with Go itself is pinned only by the reference KATs (rank_test.go:128-133:
// Pow(10,0)==1 path gives FinalScore exactly 1.0; 0.50..0.60 range).
// Must be compiled with -ffp-contract=off (no FMA contraction).
#pragma once
#include <cstdint>
#include <cstring>
#include <cmath>

namespace gomath {

static inline uint64_t bits(double x) { uint64_t u; std::memcpy(&u, &x, 8); return u; }
static inline double from_bits(uint64_t u) { double x; std::memcpy(&x, &u, 8); return x; }

static const uint64_t kMask = 0x7FF, kShift = 64 - 11 - 1, kBias = 1023;
static const uint64_t kSignMask = 1ull << 63, kFracMask = (1ull << kShift) - 1;

static inline bool is_inf(double x, int sign) {
    return (sign >= 0 && x > 1.7976931348623157e308) || (sign <= 0 && x < -1.7976931348623157e308);
}

// math.normalize (bits.go): returns a normal number y and exponent exp with x == y*2**exp.
static inline void normalize(double x, double* y, int* e) {
    const double SmallestNormal = 2.2250738585072014e-308;
    if (std::fabs(x) < SmallestNormal) { *y = x * (double)(1ull << 52); *e = -52; return; }
    *y = x; *e = 0;
}

// math.Frexp (frexp.go)
static inline double frexp(double f, int* e) {
    *e = 0;
    if (f == 0 || std::isinf(f) || std::isnan(f)) return f;
    int ne; double nf; normalize(f, &nf, &ne);
    f = nf; *e = ne;
    uint64_t x = bits(f);
    *e += (int)((x >> kShift) & kMask) - (int)kBias + 1;
    x &= ~(kMask << kShift);
    x |= (uint64_t)(-1 + (int64_t)kBias) << kShift;
    return from_bits(x);
}

// math.Ldexp (ldexp.go)
static inline double ldexp(double frac, int exp) {
    if (frac == 0) return frac;
    if (std::isinf(frac) || std::isnan(frac)) return frac;
    int e; double f; normalize(frac, &f, &e);
    exp += e;
    uint64_t x = bits(f);
    exp += (int)((x >> kShift) & kMask) - (int)kBias;
    if (exp < -1075) return std::copysign(0.0, f);
    if (exp > 1023) return f < 0 ? -INFINITY : INFINITY;
    double m = 1;
    if (exp < -1022) { exp += 53; m = 1.0 / (double)(1ull << 53); }
    x &= ~(kMask << kShift);
    x |= (uint64_t)(exp + (int)kBias) << kShift;
    return m * from_bits(x);
}

// math.Modf (modf.go): int part and fractional part with the sign of f.
static inline void modf(double f, double* ip, double* fp) {
    if (f < 1) {
        if (f < 0) { double i2, f2; modf(-f, &i2, &f2); *ip = -i2; *fp = -f2; return; }
        if (f == 0) { *ip = f; *fp = f; return; }
        *ip = 0; *fp = f; return;
    }
    uint64_t x = bits(f);
    int e = (int)((x >> kShift) & kMask) - (int)kBias;
    if (e < 64 - 12) x &= ~((1ull << (64 - 12 - e)) - 1);
    *ip = from_bits(x);
    *fp = f - *ip;
}

// math.expmulti (exp.go)
static inline double expmulti(double hi, double lo, int k) {
    const double P1 = 1.66666666666666657415e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    double r = hi - lo;
    double t = r * r;
    double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    double y = 1 - ((lo - (r * c) / (2 - c)) - hi);
    return ldexp(y, k);
}

// math.exp (exp.go)
static inline double exp(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
                 Log2e = 1.44269504088896338700e+00, Overflow = 7.09782712893383973096e+02,
                 Underflow = -7.45133219101941108420e+02, NearZero = 1.0 / (1 << 28);
    if (std::isnan(x) || (std::isinf(x) && x > 0)) return x;
    if (std::isinf(x)) return 0;
    if (x > Overflow) return INFINITY;
    if (x < Underflow) return 0;
    if (-NearZero < x && x < NearZero) return 1 + x;
    int k = 0;
    if (x < 0) k = (int)(Log2e * x - 0.5);
    else if (x > 0) k = (int)(Log2e * x + 0.5);
    double hi = x - (double)k * Ln2Hi;
    double lo = (double)k * Ln2Lo;
    return expmulti(hi, lo, k);
}

// math.log (log.go)
static inline double log(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
                 L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
                 L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
                 L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
                 L7 = 1.479819860511658591e-01;
    const double Sqrt2 = 1.41421356237309504880168872420969807856967187537694807317667974;
    if (std::isnan(x) || (std::isinf(x) && x > 0)) return x;
    if (x < 0) return NAN;
    if (x == 0) return -INFINITY;
    int ki; double f1 = frexp(x, &ki);
    if (f1 < Sqrt2 / 2) { f1 *= 2; ki--; }
    double f = f1 - 1;
    double k = (double)ki;
    double s = f / (2 + f);
    double s2 = s * s;
    double s4 = s2 * s2;
    double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
    double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
    double R = t1 + t2;
    double hfsq = 0.5 * f * f;
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

// math.pow (pow.go), finite positive x and finite y (the only domain on the
// scoring path: x = 10, y = free fraction). Special cases kept in Go's order.
static inline double pow(double x, double y) {
    if (y == 0 || x == 1) return 1;
    if (y == 1) return x;
    if (std::isnan(x) || std::isnan(y)) return NAN;
    if (x == 0) return y < 0 ? INFINITY : 0;   // (sign subtleties irrelevant for x=10)
    if (y == 0.5) return std::sqrt(x);
    if (y == -0.5) return 1 / std::sqrt(x);
    double yi, yf; modf(std::fabs(y), &yi, &yf);
    if (yf != 0 && x < 0) return NAN;
    double a1 = 1.0; int ae = 0;
    if (yf != 0) {
        if (yf > 0.5) { yf--; yi++; }
        a1 = exp(yf * log(x));
    }
    int xe; double x1 = frexp(x, &xe);
    for (int64_t i = (int64_t)yi; i != 0; i >>= 1) {
        if (xe < -(1 << 12) || (1 << 12) < xe) { ae += xe; break; }
        if (i & 1) { a1 *= x1; ae += xe; }
        x1 *= x1;
        xe <<= 1;
        if (x1 < .5) { x1 += x1; xe--; }
    }
    if (y < 0) { if (a1 != 0) a1 = 1 / a1; ae = -ae; }
    return ldexp(a1, ae);
}

}  // namespace gomath
