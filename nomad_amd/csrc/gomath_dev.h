// Device (and host) restatement of the Go 1.16 pure-Go math kernels on the
// scoring path: math.Pow(10, free) in ScoreFitBinPack / ScoreFitSpread
// (nomad/structs/funcs.go:241,267). Bit-identical to the oracle's portable
// algorithm when compiled with -ffp-contract=off.
// Domain: x = 10 (finite, positive), y = free fraction (finite).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pe {
namespace gm {

__host__ __device__ __forceinline__ uint64_t f2u(double x) {
    union { double d; uint64_t u; } v; v.d = x; return v.u;
}
__host__ __device__ __forceinline__ double u2f(uint64_t u) {
    union { double d; uint64_t u; } v; v.u = u; return v.d;
}

constexpr uint64_t kMask = 0x7FF;
constexpr int kShift = 52;
constexpr int kBias = 1023;

__host__ __device__ __forceinline__ double normalize(double x, int* e) {
    const double kSmallestNormal = 2.2250738585072014e-308;
    double ax = x < 0 ? -x : x;
    if (ax < kSmallestNormal) { *e = -52; return x * 4503599627370496.0; }
    *e = 0;
    return x;
}

__host__ __device__ __forceinline__ double frexp_go(double f, int* e) {
    *e = 0;
    if (f == 0.0) return f;
    uint64_t b = f2u(f);
    if (((b >> kShift) & kMask) == kMask) return f;   // Inf / NaN
    int ne;
    f = normalize(f, &ne);
    uint64_t x = f2u(f);
    *e = ne + (int)((x >> kShift) & kMask) - kBias + 1;
    x &= ~(kMask << kShift);
    x |= (uint64_t)(kBias - 1) << kShift;
    return u2f(x);
}

__host__ __device__ __forceinline__ double ldexp_go(double frac, int exp) {
    if (frac == 0.0) return frac;
    uint64_t b = f2u(frac);
    if (((b >> kShift) & kMask) == kMask) return frac;
    int e;
    frac = normalize(frac, &e);
    exp += e;
    uint64_t x = f2u(frac);
    exp += (int)((x >> kShift) & kMask) - kBias;
    if (exp < -1075) return (x >> 63) ? -0.0 : 0.0;
    if (exp > 1023) return (x >> 63) ? -__builtin_inf() : __builtin_inf();
    double m = 1.0;
    if (exp < -1022) { exp += 53; m = 1.0 / 9007199254740992.0; }
    x &= ~(kMask << kShift);
    x |= (uint64_t)(exp + kBias) << kShift;
    return m * u2f(x);
}

// ldexp_go for a normal frac whose result is normal: the exponent field add
// (the m == 1.0 branch of ldexp_go, bit-identical); anything else takes the
// full routine.
__host__ __device__ __forceinline__ double ldexp_fast(double frac, int exp) {
    const uint64_t x = f2u(frac);
    const int be = (int)((x >> kShift) & kMask);
    const int ne = be + exp;
    if (be != 0 && be != (int)kMask && ne > 0 && ne < (int)kMask)
        return u2f(x + ((uint64_t)(int64_t)exp << kShift));
    return ldexp_go(frac, exp);
}

// math.Modf for f >= 0
__host__ __device__ __forceinline__ void modf_go(double f, double* ip, double* fp) {
    if (f < 1.0) {
        if (f == 0.0) { *ip = f; *fp = f; return; }
        *ip = 0.0; *fp = f; return;
    }
    uint64_t x = f2u(f);
    int e = (int)((x >> kShift) & kMask) - kBias;
    if (e < 64 - 12) x &= ~((1ull << (64 - 12 - e)) - 1);
    *ip = u2f(x);
    *fp = f - *ip;
}

__host__ __device__ __forceinline__ double exp_go(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
                 Log2e = 1.44269504088896338700e+00, Overflow = 7.09782712893383973096e+02,
                 Underflow = -7.45133219101941108420e+02, NearZero = 1.0 / (1 << 28);
    const double P1 = 1.66666666666666657415e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    if (x != x) return x;
    if (x > Overflow) return __builtin_inf();
    if (x < Underflow) return 0.0;
    if (-NearZero < x && x < NearZero) return 1.0 + x;
    int k = 0;
    if (x < 0) k = (int)(Log2e * x - 0.5);
    else if (x > 0) k = (int)(Log2e * x + 0.5);
    double hi = x - (double)k * Ln2Hi;
    double lo = (double)k * Ln2Lo;
    double r = hi - lo;
    double t = r * r;
    double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    double y = 1 - ((lo - (r * c) / (2 - c)) - hi);
    return ldexp_fast(y, k);
}

__host__ __device__ __forceinline__ double log_go(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
                 L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
                 L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
                 L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
                 L7 = 1.479819860511658591e-01;
    const double Sqrt2 = 1.41421356237309504880168872420969807856967187537694807317667974;
    int ki;
    double f1 = frexp_go(x, &ki);
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

// math.Pow(10, y) with the caller's precomputed log10 = log_go(10).
// Special cases in Go's order: y == 0 -> 1, y == 1 -> x, y == 0.5 -> Sqrt(x).
__host__ __device__ __forceinline__ double pow10_go(double y, double log10) {
    const double x = 10.0;
    if (y == 0.0) return 1.0;
    if (y == 1.0) return x;
    if (y == 0.5) return __builtin_sqrt(x);
    if (y == -0.5) return 1.0 / __builtin_sqrt(x);
    double ay = y < 0 ? -y : y;
    double yi, yf;
    modf_go(ay, &yi, &yf);
    double a1 = 1.0;
    int ae = 0;
    if (yf != 0.0) {
        if (yf > 0.5) { yf -= 1.0; yi += 1.0; }
        a1 = exp_go(yf * log10);
    }
    int xe;
    double x1 = frexp_go(x, &xe);
    for (int64_t i = (int64_t)yi; i != 0; i >>= 1) {
        if (xe < -(1 << 12) || (1 << 12) < xe) { ae += xe; break; }
        if (i & 1) { a1 *= x1; ae += xe; }
        x1 *= x1;
        xe <<= 1;
        if (x1 < 0.5) { x1 += x1; xe--; }
    }
    if (y < 0) {
        if (a1 != 0.0) a1 = 1.0 / a1;
        ae = -ae;
    }
    return ldexp_go(a1, ae);
}

// pow10_go on the free fractions ScoreFit sees (0 < y < 1, y != 0.5): Modf
// gives yi = 0, and for yf > 0.5 the shifted fraction yf - 1 with yi = 1, whose
// one loop step multiplies by Frexp(10) = 0.625 * 2^4. The same operations in
// the same order as pow10_go, without the loop; other y take pow10_go.
// exp_go restricted to |x| < 2: NaN / overflow / underflow cannot occur, the
// reduction gives |k| <= 3 and y in (0.7, 1.5), so the closing ldexp_go is the
// exponent-field add (its m == 1.0 branch).
__host__ __device__ __forceinline__ double exp_small(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
                 Log2e = 1.44269504088896338700e+00, NearZero = 1.0 / (1 << 28);
    const double P1 = 1.66666666666666657415e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    if (-NearZero < x && x < NearZero) return 1.0 + x;
    const int k = (int)(x < 0 ? Log2e * x - 0.5 : Log2e * x + 0.5);
    double hi = x - (double)k * Ln2Hi;
    double lo = (double)k * Ln2Lo;
    double r = hi - lo;
    double t = r * r;
    double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    double y = 1 - ((lo - (r * c) / (2 - c)) - hi);
    return u2f(f2u(y) + ((uint64_t)(int64_t)k << kShift));
}

__host__ __device__ __forceinline__ double pow10_unit(double y, double log10) {
    if (y > 0.0 && y < 1.0 && y != 0.5) {
        // (y - 1) * log10 in (-1.16, 0): exp in (0.31, 1), times 0.625 stays
        // normal, so ldexp_go(., 4) is the exponent add as well
        if (y > 0.5) return u2f(f2u(exp_small((y - 1.0) * log10) * 0.625) + (4ull << kShift));
        return exp_small(y * log10);
    }
    return pow10_go(y, log10);
}

// ScoreFitBinPack / ScoreFitSpread (funcs.go:237-279) divided by
// binPackingMaxFitScore (rank.go:514).
__host__ __device__ __forceinline__ double fit_score(int64_t cap_cpu, int64_t cap_mem, int64_t util_cpu,
                                                     int64_t util_mem, int spread, double log10) {
    const double node_cpu = (double)cap_cpu, node_mem = (double)cap_mem;
    const double fc = 1 - ((double)util_cpu / node_cpu);
    const double fm = 1 - ((double)util_mem / node_mem);
    const double total = pow10_unit(fc, log10) + pow10_unit(fm, log10);
    double s = spread ? total - 2 : 20.0 - total;
    if (s > 18.0) s = 18.0;
    else if (s < 0) s = 0;
    return s / 18.0;
}

}  // namespace gm
}  // namespace pe
