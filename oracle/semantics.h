// ORACLE — test infrastructure only (never linked into the product).
//
// Restatement of the constraint semantics the placement stack evaluates per node:
//   checkConstraint / checkLexicalOrder / checkVersionMatch / checkRegexpMatch /
//   checkSetContainsAll / checkSetContainsAny   (scheduler/feasible.go:785-1024)
//   github.com/hashicorp/go-version @ v1.2.1-0.20191009193637-2046c9d0f0b0
//     (go.mod:75; not vendored in the reference): NewVersion/NewSemver, Compare,
//     comparePrereleases, Constraint operators incl. prereleaseCheck and "~>".
//   helper/constraints/semver/constraints.go (semver operand: Semver 2.0 ordering,
//     no "~>" operator).
// Regexp: Go 1.16's regexp package (RE2 syntax) is restated in go_regexp.h.
#pragma once
#include <cstdint>
#include <string>
#include <vector>
#include <regex>
#include <cstring>
#include <cmath>
#include <algorithm>
#include <map>
#include <memory>
#include <cctype>
#include <climits>

#include "go_regexp.h"

namespace orasem {

// A resolved target: Go's (interface{}, bool). `nil` only for unknown ${...}
// interpolations (feasible.go:778-779); a missing attribute resolves to ("", false).
struct Val {
    bool is_nil = true;
    std::string s;
};

static inline bool deep_equal(const Val& a, const Val& b) {
    if (a.is_nil || b.is_nil) return a.is_nil && b.is_nil;
    return a.s == b.s;
}

// ---------------- go-version ----------------
struct Version {
    std::vector<int64_t> segments;  // padded to >= 3
    int si = 0;                     // number of specified segments
    std::string pre, metadata, original;
};

static inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
static inline bool is_ident(char c) {   // [0-9A-Za-z\-~]
    return std::isalnum((unsigned char)c) || c == '-' || c == '~';
}

// parse int64 like strconv.ParseInt(s, 10, 64)
static inline bool parse_i64(const std::string& s, int64_t* out) {
    if (s.empty()) return false;
    size_t i = 0; bool neg = false;
    if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; if (s.size() == 1) return false; }
    __int128 v = 0;
    for (; i < s.size(); i++) {
        if (!is_digit(s[i])) return false;
        v = v * 10 + (s[i] - '0');
        if (v > (__int128)INT64_MAX + 1) return false;
    }
    if (neg) v = -v;
    if (v > INT64_MAX || v < INT64_MIN) return false;
    *out = (int64_t)v;
    return true;
}

// dotted identifier list: ident(.ident)*  where the first ident obeys `first`
static inline size_t match_dotted(const std::string& s, size_t p) {
    size_t q = p;
    if (q >= s.size() || !is_ident(s[q])) return std::string::npos;
    while (q < s.size() && is_ident(s[q])) q++;
    while (q < s.size() && s[q] == '.') {
        size_t r = q + 1;
        if (r >= s.size() || !is_ident(s[r])) break;
        while (r < s.size() && is_ident(s[r])) r++;
        q = r;
    }
    return q;
}

static inline const std::regex& version_re(bool semver) {
    // Both patterns share one group layout (go-version version.go): 1 segments,
    // 4 numeric-led prerelease, 7 alpha-led prerelease, 10 metadata. Semver
    // requires the '-' before an alpha-led prerelease ("1.0beta1" is invalid).
    static const std::regex v(
        "^v?([0-9]+(\\.[0-9]+)*?)"
        "(-([0-9]+[0-9A-Za-z\\-~]*(\\.[0-9A-Za-z\\-~]+)*)|(-?([A-Za-z\\-~]+[0-9A-Za-z\\-~]*(\\.[0-9A-Za-z\\-~]+)*)))?"
        "(\\+([0-9A-Za-z\\-~]+(\\.[0-9A-Za-z\\-~]+)*))?$");
    static const std::regex sv(
        "^v?([0-9]+(\\.[0-9]+)*?)"
        "(-([0-9]+[0-9A-Za-z\\-~]*(\\.[0-9A-Za-z\\-~]+)*)|(-([A-Za-z\\-~]+[0-9A-Za-z\\-~]*(\\.[0-9A-Za-z\\-~]+)*)))?"
        "(\\+([0-9A-Za-z\\-~]+(\\.[0-9A-Za-z\\-~]+)*))?$");
    return semver ? sv : v;
}

static inline bool new_version(const std::string& s, bool semver, Version* out) {
    std::smatch m;
    if (!std::regex_match(s, m, version_re(semver))) return false;
    std::string segs = m[1].str();
    Version v;
    size_t start = 0;
    while (true) {
        size_t dot = segs.find('.', start);
        std::string part = segs.substr(start, dot == std::string::npos ? std::string::npos : dot - start);
        int64_t x;
        if (!parse_i64(part, &x)) return false;
        v.segments.push_back(x);
        if (dot == std::string::npos) break;
        start = dot + 1;
    }
    v.si = (int)v.segments.size();
    while (v.segments.size() < 3) v.segments.push_back(0);
    v.pre = m[7].matched ? m[7].str() : "";
    if (v.pre.empty() && m[4].matched) v.pre = m[4].str();
    v.metadata = m[10].matched ? m[10].str() : "";
    v.original = s;
    *out = v;
    return true;
}

static inline std::string version_string(const Version& v) {
    std::string o;
    for (size_t i = 0; i < v.segments.size(); i++) {
        if (i) o += ".";
        o += std::to_string(v.segments[i]);
    }
    if (!v.pre.empty()) o += "-" + v.pre;
    if (!v.metadata.empty()) o += "+" + v.metadata;
    return o;
}

static inline int compare_part(const std::string& a, const std::string& b) {
    if (a == b) return 0;
    int64_t ai = 0, bi = 0;
    bool an = parse_i64(a, &ai), bn = parse_i64(b, &bi);
    if (a.empty()) return bn ? -1 : 1;
    if (b.empty()) return an ? 1 : -1;
    if (an && !bn) return -1;
    if (!an && bn) return 1;
    if (!an && !bn && a > b) return 1;
    if (ai > bi) return 1;
    return -1;
}

static inline std::vector<std::string> split(const std::string& s, char sep) {
    std::vector<std::string> out;
    size_t start = 0;
    while (true) {
        size_t p = s.find(sep, start);
        out.push_back(s.substr(start, p == std::string::npos ? std::string::npos : p - start));
        if (p == std::string::npos) break;
        start = p + 1;
    }
    return out;
}

static inline int compare_prereleases(const std::string& a, const std::string& b) {
    if (a == b) return 0;
    auto as = split(a, '.'), bs = split(b, '.');
    size_t n = std::max(as.size(), bs.size());
    for (size_t i = 0; i < n; i++) {
        std::string pa = i < as.size() ? as[i] : "";
        std::string pb = i < bs.size() ? bs[i] : "";
        int c = compare_part(pa, pb);
        if (c != 0) return c;
    }
    return 0;
}

static inline bool all_zero(const std::vector<int64_t>& s, size_t from) {
    for (size_t i = from; i < s.size(); i++) if (s[i] != 0) return false;
    return true;
}

static inline int version_compare(const Version& v, const Version& o) {
    if (version_string(v) == version_string(o)) return 0;
    if (v.segments == o.segments) {
        if (v.pre.empty() && o.pre.empty()) return 0;
        if (v.pre.empty()) return 1;
        if (o.pre.empty()) return -1;
        return compare_prereleases(v.pre, o.pre);
    }
    size_t ls = v.segments.size(), lo = o.segments.size();
    size_t hs = std::max(ls, lo);
    for (size_t i = 0; i < hs; i++) {
        if (i > ls - 1) { if (!all_zero(o.segments, i)) return -1; break; }
        if (i > lo - 1) { if (!all_zero(v.segments, i)) return 1; break; }
        int64_t l = v.segments[i], r = o.segments[i];
        if (l == r) continue;
        return l < r ? -1 : 1;
    }
    return 0;
}

enum Op { OP_EQ, OP_NE, OP_GT, OP_LT, OP_GE, OP_LE, OP_PESS };
struct VConstraint { Op op; Version check; };

static inline bool prerelease_check(const Version& v, const Version& c) {
    bool vp = !v.pre.empty(), cp = !c.pre.empty();
    if (cp && vp) return c.segments == v.segments;
    if (!cp && vp) return false;
    return true;
}

static inline bool vconstraint_check(const VConstraint& c, const Version& v, bool semver) {
    int cmp;
    switch (c.op) {
        case OP_EQ: return version_compare(v, c.check) == 0;
        case OP_NE: return version_compare(v, c.check) != 0;
        default: break;
    }
    if (!semver && !prerelease_check(v, c.check)) return false;
    switch (c.op) {
        case OP_GT: return version_compare(v, c.check) == 1;
        case OP_LT: return version_compare(v, c.check) == -1;
        case OP_GE: return version_compare(v, c.check) >= 0;
        case OP_LE: return version_compare(v, c.check) <= 0;
        case OP_PESS: {
            if (!c.check.pre.empty() && v.pre.empty()) return false;
            cmp = version_compare(v, c.check);
            if (cmp == -1) return false;
            size_t cs = c.check.segments.size();
            if (cs > v.segments.size()) return false;
            for (int i = 0; i < c.check.si - 1; i++)
                if (v.segments[i] != c.check.segments[i]) return false;
            if (c.check.segments[cs - 1] > v.segments[cs - 1]) return false;
            return true;
        }
        default: return false;
    }
}

static inline std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) a++;
    while (b > a && std::isspace((unsigned char)s[b - 1])) b--;
    return s.substr(a, b - a);
}

// version.NewConstraint / semver.NewConstraint: `^\s*(op)\s*(version)\s*$`
static inline bool parse_constraints(const std::string& str, bool semver, std::vector<VConstraint>* out) {
    out->clear();
    for (const std::string& raw : split(str, ',')) {
        std::string s = trim(raw);
        Op op = OP_EQ; size_t p = 0;
        if (!semver && s.compare(0, 2, "~>") == 0) { op = OP_PESS; p = 2; }
        else if (s.compare(0, 2, ">=") == 0) { op = OP_GE; p = 2; }
        else if (s.compare(0, 2, "<=") == 0) { op = OP_LE; p = 2; }
        else if (s.compare(0, 2, "!=") == 0) { op = OP_NE; p = 2; }
        else if (s.compare(0, 1, ">") == 0) { op = OP_GT; p = 1; }
        else if (s.compare(0, 1, "<") == 0) { op = OP_LT; p = 1; }
        else if (s.compare(0, 1, "=") == 0) { op = OP_EQ; p = 1; }
        std::string vs = trim(s.substr(p));
        Version v;
        if (!new_version(vs, semver, &v)) return false;
        out->push_back(VConstraint{op, v});
    }
    return true;
}

struct Caches {
    struct Compiled { bool ok = false; std::vector<orare::Re> pool; int root = 0; };
    std::map<std::string, std::shared_ptr<Compiled>> re;
    std::map<std::string, std::shared_ptr<std::vector<VConstraint>>> ver, semver;
};

// checkVersionMatch (feasible.go:860-892); lVal int case is unreachable for
// node attributes (they are strings).
static inline bool check_version_match(Caches& c, bool semver, const Val& l, const Val& r) {
    if (l.is_nil) return false;
    Version v;
    if (!new_version(l.s, false, &v)) return false;
    if (r.is_nil) return false;
    auto& cache = semver ? c.semver : c.ver;
    auto it = cache.find(r.s);
    std::shared_ptr<std::vector<VConstraint>> cs;
    if (it != cache.end()) cs = it->second;
    else {
        auto p = std::make_shared<std::vector<VConstraint>>();
        if (!parse_constraints(r.s, semver, p.get())) return false;
        cache[r.s] = p; cs = p;
    }
    for (auto& k : *cs) if (!vconstraint_check(k, v, semver)) return false;
    return true;
}

// checkRegexpMatch (feasible.go:931-960)
static inline bool check_regexp_match(Caches& c, const Val& l, const Val& r) {
    if (l.is_nil || r.is_nil) return false;
    auto it = c.re.find(r.s);
    if (it == c.re.end()) {
        auto k = std::make_shared<Caches::Compiled>();
        k->ok = orare::compile(r.s, &k->pool, &k->root);
        it = c.re.emplace(r.s, k).first;
    }
    return it->second->ok && orare::match_string(it->second->pool, it->second->root, l.s);
}

static inline bool check_set_contains_all(const Val& l, const Val& r) {
    if (l.is_nil || r.is_nil) return false;
    std::map<std::string, int> lookup;
    for (auto& in : split(l.s, ',')) lookup[trim(in)] = 1;
    for (auto& x : split(r.s, ',')) if (!lookup.count(trim(x))) return false;
    return true;
}

static inline bool check_set_contains_any(const Val& l, const Val& r) {
    if (l.is_nil || r.is_nil) return false;
    std::map<std::string, int> lookup;
    for (auto& in : split(l.s, ',')) lookup[trim(in)] = 1;
    for (auto& x : split(r.s, ',')) if (lookup.count(trim(x))) return true;
    return false;
}

static inline bool check_lexical_order(const std::string& op, const Val& l, const Val& r) {
    if (l.is_nil || r.is_nil) return false;
    if (op == "<") return l.s < r.s;
    if (op == "<=") return l.s <= r.s;
    if (op == ">") return l.s > r.s;
    if (op == ">=") return l.s >= r.s;
    return false;
}

// checkConstraint (feasible.go:785-820)
static inline bool check_constraint(Caches& c, const std::string& op, const Val& l, const Val& r,
                                    bool lf, bool rf) {
    if (op == "distinct_hosts" || op == "distinct_property") return true;
    if (op == "=" || op == "==" || op == "is") return lf && rf && deep_equal(l, r);
    if (op == "!=" || op == "not") return !deep_equal(l, r);
    if (op == "<" || op == "<=" || op == ">" || op == ">=") return lf && rf && check_lexical_order(op, l, r);
    if (op == "is_set") return lf;
    if (op == "is_not_set") return !lf;
    if (op == "version") return lf && rf && check_version_match(c, false, l, r);
    if (op == "semver") return lf && rf && check_version_match(c, true, l, r);
    if (op == "regexp") return lf && rf && check_regexp_match(c, l, r);
    if (op == "set_contains" || op == "set_contains_all") return lf && rf && check_set_contains_all(l, r);
    if (op == "set_contains_any") return lf && rf && check_set_contains_any(l, r);
    return false;
}

// ---------------- device attributes ----------------
// plugins/shared/structs/attribute.go (ParseAttribute 55-103, Comparable 296-320,
// Compare 322-385) and units.go (unit table); checkAttributeConstraint and
// checkAttributeVersionMatch (scheduler/feasible.go:1334-1447, 896-930).
// Numbers are compared through long double where Go uses a 256-bit big.Float:
// exact whenever value bits + multiplier bits <= 64 (every unit multiplier here
// is <= 2^60 or 10^18; beyond that the comparison is parity unpinned).
struct Attr {
    enum Kind { None, Int, Float, Str, Bool } kind = None;
    int64_t i = 0;
    double f = 0;
    std::string s;
    bool b = false;
    std::string unit;
};

struct UnitDef { const char* name; int base; int64_t mult; bool inverse; };
static inline const std::vector<UnitDef>& unit_table() {
    static const std::vector<UnitDef> t = {
        {"KiB", 1, 1ll << 10, false}, {"MiB", 1, 1ll << 20, false}, {"GiB", 1, 1ll << 30, false},
        {"TiB", 1, 1ll << 40, false}, {"PiB", 1, 1ll << 50, false}, {"EiB", 1, 1ll << 60, false},
        {"kB", 1, 1000ll, false}, {"KB", 1, 1000ll, false}, {"MB", 1, 1000000ll, false},
        {"GB", 1, 1000000000ll, false}, {"TB", 1, 1000000000000ll, false},
        {"PB", 1, 1000000000000000ll, false}, {"EB", 1, 1000000000000000000ll, false},
        {"KiB/s", 2, 1ll << 10, false}, {"MiB/s", 2, 1ll << 20, false}, {"GiB/s", 2, 1ll << 30, false},
        {"TiB/s", 2, 1ll << 40, false}, {"PiB/s", 2, 1ll << 50, false}, {"EiB/s", 2, 1ll << 60, false},
        {"kB/s", 2, 1000ll, false}, {"KB/s", 2, 1000ll, false}, {"MB/s", 2, 1000000ll, false},
        {"GB/s", 2, 1000000000ll, false}, {"TB/s", 2, 1000000000000ll, false},
        {"PB/s", 2, 1000000000000000ll, false}, {"EB/s", 2, 1000000000000000000ll, false},
        {"MHz", 3, 1000000ll, false}, {"GHz", 3, 1000000000ll, false},
        {"mW", 4, 1000ll, true}, {"W", 4, 1ll, false}, {"kW", 4, 1000ll, false},
        {"MW", 4, 1000000ll, false}, {"GW", 4, 1000000000ll, false},
    };
    return t;
}
static inline const UnitDef* find_unit(const std::string& u) {
    if (u.empty()) return nullptr;
    for (auto& d : unit_table()) if (u == d.name) return &d;
    return nullptr;
}

static inline std::string trim_space(const std::string& x) {
    size_t a = 0, b = x.size();
    while (a < b && std::isspace((unsigned char)x[a])) a++;
    while (b > a && std::isspace((unsigned char)x[b - 1])) b--;
    return x.substr(a, b - a);
}

// strconv.ParseFloat(s, 64) for the decimal forms (sign, digits, '.', exponent,
// inf/infinity/nan)
static inline bool parse_f64(const std::string& x, double* out) {
    if (x.empty()) return false;
    std::string l;
    for (char c : x) l += (char)std::tolower((unsigned char)c);
    size_t p = (l[0] == '+' || l[0] == '-') ? 1 : 0;
    std::string body = l.substr(p);
    if (body == "inf" || body == "infinity") { *out = l[0] == '-' ? -HUGE_VAL : HUGE_VAL; return true; }
    if (body == "nan" && p == 0) { *out = NAN; return true; }
    bool digits = false, dot = false;
    size_t i = p;
    for (; i < l.size(); i++) {
        if (is_digit(l[i])) digits = true;
        else if (l[i] == '.' && !dot) dot = true;
        else break;
    }
    if (!digits) return false;
    if (i < l.size() && l[i] == 'e') {
        i++;
        if (i < l.size() && (l[i] == '+' || l[i] == '-')) i++;
        bool ed = false;
        while (i < l.size() && is_digit(l[i])) { i++; ed = true; }
        if (!ed) return false;
    }
    if (i != l.size()) return false;
    *out = std::strtod(x.c_str(), nullptr);
    return true;
}

// psstructs.ParseAttribute (attribute.go:55-103)
static inline Attr parse_attribute(const std::string& in) {
    Attr a;
    if (in.empty()) { a.kind = Attr::Str; return a; }
    std::string unit, numeric = in;
    if (std::isalpha((unsigned char)in.back())) {
        // lengthSortedUnits: longest unit first
        std::vector<const UnitDef*> us;
        for (auto& d : unit_table()) us.push_back(&d);
        std::stable_sort(us.begin(), us.end(), [](const UnitDef* x, const UnitDef* y) {
            return std::strlen(x->name) > std::strlen(y->name);
        });
        for (auto* d : us) {
            const size_t n = std::strlen(d->name);
            if (in.size() >= n && in.compare(in.size() - n, n, d->name) == 0) { unit = d->name; break; }
        }
        if (!unit.empty()) numeric = trim_space(in.substr(0, in.size() - unit.size()));
    }
    int64_t iv;
    if (parse_i64(numeric, &iv)) { a.kind = Attr::Int; a.i = iv; a.unit = unit; return a; }
    double fv;
    if (parse_f64(numeric, &fv)) { a.kind = Attr::Float; a.f = fv; a.unit = unit; return a; }
    static const char* tr[] = {"1", "t", "T", "TRUE", "true", "True"};
    static const char* fa[] = {"0", "f", "F", "FALSE", "false", "False"};
    for (auto* t : tr) if (in == t) { a.kind = Attr::Bool; a.b = true; return a; }
    for (auto* t : fa) if (in == t) { a.kind = Attr::Bool; a.b = false; return a; }
    a.kind = Attr::Str; a.s = in;
    return a;
}

static inline bool attr_comparable(const Attr& a, const Attr& b) {
    const UnitDef* ua = find_unit(a.unit);
    const UnitDef* ub = find_unit(b.unit);
    if (ua && ub) return ua->base == ub->base;
    if (ua || ub) return false;
    if (a.kind == Attr::Str) return b.kind == Attr::Str;
    if (a.kind == Attr::Bool) return b.kind == Attr::Bool;
    return true;
}

// Attribute.Compare (attribute.go:322-385)
static inline int attr_compare(const Attr& a, const Attr& b, bool* ok) {
    *ok = false;
    if (!attr_comparable(a, b)) return 0;
    if (a.kind == Attr::Bool) { *ok = true; return a.b == b.b ? 0 : 1; }
    if (a.kind == Attr::Str) { *ok = true; return a.s < b.s ? -1 : (a.s == b.s ? 0 : 1); }
    if (a.kind != Attr::Int && a.kind != Attr::Float) return 0;   // nullComparator
    if (a.kind == Attr::Int && b.kind == Attr::Int) {
        auto scaled = [](const Attr& x) -> int64_t {   // getInt: int64 arithmetic (wraps like Go)
            const UnitDef* u = find_unit(x.unit);
            if (!u) return x.i;
            if (u->inverse) return x.i / u->mult;
            return (int64_t)((uint64_t)x.i * (uint64_t)u->mult);
        };
        const int64_t ai = scaled(a), bi = scaled(b);
        *ok = true;
        return ai == bi ? 0 : (ai < bi ? -1 : 1);
    }
    if (b.kind != Attr::Int && b.kind != Attr::Float) return 0;
    auto big = [](const Attr& x) -> long double {
        long double v = x.kind == Attr::Int ? (long double)x.i : (long double)x.f;
        const UnitDef* u = find_unit(x.unit);
        if (!u) return v;
        return u->inverse ? v * (1.0L / (long double)u->mult) : v * (long double)u->mult;
    };
    const long double af = big(a), bf = big(b);
    *ok = true;
    return af < bf ? -1 : (af > bf ? 1 : 0);
}

// checkAttributeVersionMatch (feasible.go:896-930)
static inline bool check_attr_version(Caches& c, bool semver, const Attr& l, const Attr& r) {
    std::string vs;
    if (l.kind == Attr::Str) vs = l.s;
    else if (l.kind == Attr::Int) vs = std::to_string(l.i);
    else return false;
    if (r.kind != Attr::Str) return false;
    Val lv, rv;
    lv.is_nil = false; lv.s = vs;
    rv.is_nil = false; rv.s = r.s;
    return check_version_match(c, semver, lv, rv);
}

// checkAttributeConstraint (feasible.go:1334-1447)
static inline bool check_attribute_constraint(Caches& c, const std::string& op, const Attr& l, const Attr& r,
                                              bool lf, bool rf) {
    if (op == "distinct_hosts" || op == "distinct_property") return true;
    if (op == "!=" || op == "not") {
        if (!(lf || rf)) return false;
        if (lf != rf) return true;
        bool ok;
        int v = attr_compare(l, r, &ok);
        return ok && v != 0;
    }
    if (op == "<" || op == "<=" || op == ">" || op == ">=" || op == "=" || op == "==" || op == "is") {
        if (!(lf && rf)) return false;
        bool ok;
        int v = attr_compare(l, r, &ok);
        if (!ok) return false;
        if (op == "is" || op == "==" || op == "=") return v == 0;
        if (op == "<") return v == -1;
        if (op == "<=") return v != 1;
        if (op == ">") return v == 1;
        return v != -1;
    }
    if (op == "version" || op == "semver") return lf && rf && check_attr_version(c, op == "semver", l, r);
    if (op == "regexp" || op == "set_contains" || op == "set_contains_all" || op == "set_contains_any") {
        if (!(lf && rf) || l.kind != Attr::Str || r.kind != Attr::Str) return false;
        Val lv, rv;
        lv.is_nil = false; lv.s = l.s;
        rv.is_nil = false; rv.s = r.s;
        if (op == "regexp") return check_regexp_match(c, lv, rv);
        if (op == "set_contains_any") return check_set_contains_any(lv, rv);
        return check_set_contains_all(lv, rv);
    }
    if (op == "is_set") return lf;
    if (op == "is_not_set") return !lf;
    return false;
}

}  // namespace orasem
