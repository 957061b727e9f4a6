// Host-side constraint semantics (see constraint_eval.h).
#include "constraint_eval.h"
#include <cmath>
#include <cstring>

#include <algorithm>
#include <cctype>
#include <climits>

namespace pe {

namespace {

inline bool ident_char(char c) { return std::isalnum((unsigned char)c) || c == '-' || c == '~'; }
inline bool alpha_lead(char c) { return std::isalpha((unsigned char)c) || c == '-' || c == '~'; }
inline bool digit(char c) { return c >= '0' && c <= '9'; }

// strconv.ParseInt(s, 10, 64)
bool to_i64(const std::string& s, int64_t* out) {
    if (s.empty()) return false;
    size_t i = 0;
    bool neg = false;
    if (s[0] == '+' || s[0] == '-') {
        neg = s[0] == '-';
        if (s.size() == 1) return false;
        i = 1;
    }
    unsigned long long acc = 0;
    const unsigned long long lim = neg ? (unsigned long long)INT64_MAX + 1ull : (unsigned long long)INT64_MAX;
    for (; i < s.size(); i++) {
        if (!digit(s[i])) return false;
        unsigned d = (unsigned)(s[i] - '0');
        if (acc > (lim - d) / 10) return false;
        acc = acc * 10 + d;
    }
    *out = neg ? (int64_t)(0 - acc) : (int64_t)acc;
    return true;
}

// ident+ ('.' ident+)* starting at p (first char already validated by caller
// as part of an ident run). Returns the end position.
size_t scan_dotted(const std::string& s, size_t p) {
    while (p < s.size() && ident_char(s[p])) p++;
    while (p + 1 < s.size() && s[p] == '.' && ident_char(s[p + 1])) {
        p++;
        while (p < s.size() && ident_char(s[p])) p++;
    }
    return p;
}

std::vector<std::string> split_on(const std::string& s, char sep) {
    std::vector<std::string> out;
    size_t b = 0;
    for (;;) {
        size_t e = s.find(sep, b);
        out.emplace_back(s, b, e == std::string::npos ? std::string::npos : e - b);
        if (e == std::string::npos) return out;
        b = e + 1;
    }
}

std::string strip(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) a++;
    while (b > a && std::isspace((unsigned char)s[b - 1])) b--;
    return s.substr(a, b - a);
}

int cmp_pre_part(const std::string& a, const std::string& b) {
    if (a == b) return 0;
    int64_t ai = 0, bi = 0;
    const bool an = to_i64(a, &ai), bn = to_i64(b, &bi);
    if (a.empty()) return bn ? -1 : 1;
    if (b.empty()) return an ? 1 : -1;
    if (an != bn) return an ? -1 : 1;
    if (!an) return a > b ? 1 : -1;
    return ai > bi ? 1 : -1;
}

std::string canonical(const SemVer& v) {
    std::string o;
    for (size_t i = 0; i < v.seg.size(); i++) {
        if (i) o.push_back('.');
        o += std::to_string(v.seg[i]);
    }
    if (!v.pre.empty()) o += "-" + v.pre;
    if (!v.meta.empty()) o += "+" + v.meta;
    return o;
}

}  // namespace

bool parse_version(const std::string& s, bool semver, SemVer* out) {
    size_t p = 0;
    if (p < s.size() && s[p] == 'v') p++;
    // segments: [0-9]+ ('.' [0-9]+)*
    size_t seg_begin = p;
    if (p >= s.size() || !digit(s[p])) return false;
    while (p < s.size() && digit(s[p])) p++;
    while (p + 1 < s.size() && s[p] == '.' && digit(s[p + 1])) {
        p++;
        while (p < s.size() && digit(s[p])) p++;
    }
    const std::string segs = s.substr(seg_begin, p - seg_begin);
    std::string pre;
    if (p < s.size() && s[p] != '+') {
        if (s[p] == '-' && p + 1 < s.size() && digit(s[p + 1])) {
            // numeric-led prerelease (group 4)
            size_t e = scan_dotted(s, p + 1);
            pre = s.substr(p + 1, e - p - 1);
            p = e;
        } else if (s[p] == '-' && p + 1 < s.size() && alpha_lead(s[p + 1])) {
            size_t e = scan_dotted(s, p + 1);
            pre = s.substr(p + 1, e - p - 1);
            p = e;
        } else if (!semver && alpha_lead(s[p])) {
            // '-?' matched empty: the run starts at p (may itself be '-')
            size_t e = scan_dotted(s, p);
            pre = s.substr(p, e - p);
            p = e;
        } else {
            return false;
        }
    }
    std::string meta;
    if (p < s.size() && s[p] == '+') {
        if (p + 1 >= s.size() || !ident_char(s[p + 1])) return false;
        size_t e = scan_dotted(s, p + 1);
        meta = s.substr(p + 1, e - p - 1);
        p = e;
    }
    if (p != s.size()) return false;
    SemVer v;
    for (const std::string& part : split_on(segs, '.')) {
        int64_t x;
        if (!to_i64(part, &x)) return false;
        v.seg.push_back(x);
    }
    v.specified = (int)v.seg.size();
    while (v.seg.size() < 3) v.seg.push_back(0);
    v.pre = pre;
    v.meta = meta;
    *out = v;
    return true;
}

int compare_versions(const SemVer& a, const SemVer& b) {
    if (canonical(a) == canonical(b)) return 0;
    if (a.seg == b.seg) {
        if (a.pre.empty() && b.pre.empty()) return 0;
        if (a.pre.empty()) return 1;
        if (b.pre.empty()) return -1;
        if (a.pre == b.pre) return 0;
        auto pa = split_on(a.pre, '.'), pb = split_on(b.pre, '.');
        const size_t n = std::max(pa.size(), pb.size());
        for (size_t i = 0; i < n; i++) {
            int c = cmp_pre_part(i < pa.size() ? pa[i] : std::string(), i < pb.size() ? pb[i] : std::string());
            if (c) return c;
        }
        return 0;
    }
    const size_t la = a.seg.size(), lb = b.seg.size(), hs = std::max(la, lb);
    for (size_t i = 0; i < hs; i++) {
        if (i >= la) {
            for (size_t k = i; k < lb; k++) if (b.seg[k] != 0) return -1;
            return 0;
        }
        if (i >= lb) {
            for (size_t k = i; k < la; k++) if (a.seg[k] != 0) return 1;
            return 0;
        }
        if (a.seg[i] != b.seg[i]) return a.seg[i] < b.seg[i] ? -1 : 1;
    }
    return 0;
}

bool parse_version_constraints(const std::string& s, bool semver, std::vector<VersionConstraint>* out) {
    static const struct { const char* tok; int op; } kOps[] = {
        {"~>", 6}, {">=", 4}, {"<=", 5}, {"!=", 1}, {">", 2}, {"<", 3}, {"=", 0}};
    out->clear();
    for (const std::string& raw : split_on(s, ',')) {
        std::string t = strip(raw);
        int op = 0;
        size_t skip = 0;
        for (const auto& o : kOps) {
            const size_t L = std::char_traits<char>::length(o.tok);
            if (t.compare(0, L, o.tok) == 0) {
                if (o.op == 6 && semver) return false;   // semver has no pessimistic operator
                op = o.op;
                skip = L;
                break;
            }
        }
        VersionConstraint c;
        c.op = op;
        if (!parse_version(strip(t.substr(skip)), semver, &c.v)) return false;
        out->push_back(c);
    }
    return true;
}

static bool prerelease_ok(const SemVer& v, const SemVer& c) {
    const bool vp = !v.pre.empty(), cp = !c.pre.empty();
    if (cp && vp) return c.seg == v.seg;
    if (!cp && vp) return false;
    return true;
}

bool check_version_constraints(const std::vector<VersionConstraint>& cs, const SemVer& v, bool semver) {
    for (const auto& c : cs) {
        bool ok;
        switch (c.op) {
            case 0: ok = compare_versions(v, c.v) == 0; break;
            case 1: ok = compare_versions(v, c.v) != 0; break;
            case 2: ok = (semver || prerelease_ok(v, c.v)) && compare_versions(v, c.v) == 1; break;
            case 3: ok = (semver || prerelease_ok(v, c.v)) && compare_versions(v, c.v) == -1; break;
            case 4: ok = (semver || prerelease_ok(v, c.v)) && compare_versions(v, c.v) >= 0; break;
            case 5: ok = (semver || prerelease_ok(v, c.v)) && compare_versions(v, c.v) <= 0; break;
            case 6: {
                ok = prerelease_ok(v, c.v) && !(!c.v.pre.empty() && v.pre.empty());
                if (ok && compare_versions(v, c.v) == -1) ok = false;
                const size_t cs_len = c.v.seg.size();
                if (ok && cs_len > v.seg.size()) ok = false;
                for (int i = 0; ok && i < c.v.specified - 1; i++)
                    if (v.seg[i] != c.v.seg[i]) ok = false;
                if (ok && c.v.seg[cs_len - 1] > v.seg[cs_len - 1]) ok = false;
                break;
            }
            default: ok = false;
        }
        if (!ok) return false;
    }
    return true;
}

bool ConstraintEvaluator::version_match(bool semver, const Target& l, const Target& r) {
    if (l.nil || r.nil) return false;
    SemVer v;
    if (!parse_version(l.value, false, &v)) return false;
    auto& cache = ver_cache_[semver ? 1 : 0];
    auto it = cache.find(r.value);
    if (it == cache.end()) {
        auto cs = std::make_shared<std::vector<VersionConstraint>>();
        if (!parse_version_constraints(r.value, semver, cs.get())) return false;
        it = cache.emplace(r.value, cs).first;
    }
    return check_version_constraints(*it->second, v, semver);
}

// checkRegexpMatch (feasible.go:931-960): Go's regexp (RE2 syntax), see go_regexp.h.
bool ConstraintEvaluator::regexp_match(const Target& l, const Target& r) {
    if (l.nil || r.nil) return false;
    auto it = re_cache_.find(r.value);
    if (it == re_cache_.end()) {
        int status;
        it = re_cache_.emplace(r.value, gore::compile(r.value, &status)).first;
    }
    return it->second && gore::match(*it->second, l.value);
}

static bool set_contains(const Target& l, const Target& r, bool all) {
    if (l.nil || r.nil) return false;
    std::vector<std::string> have;
    for (auto& x : split_on(l.value, ',')) have.push_back(strip(x));
    std::sort(have.begin(), have.end());
    for (auto& x : split_on(r.value, ',')) {
        const bool in = std::binary_search(have.begin(), have.end(), strip(x));
        if (all && !in) return false;
        if (!all && in) return true;
    }
    return all;
}

static bool same(const Target& a, const Target& b) {   // reflect.DeepEqual on resolved values
    if (a.nil || b.nil) return a.nil && b.nil;
    return a.value == b.value;
}

bool ConstraintEvaluator::check(const std::string& op, const Target& l, const Target& r) {
    if (op == "distinct_hosts" || op == "distinct_property") return true;
    if (op == "=" || op == "==" || op == "is") return l.found && r.found && same(l, r);
    if (op == "!=" || op == "not") return !same(l, r);
    if (op == "<" || op == "<=" || op == ">" || op == ">=") {
        if (!(l.found && r.found) || l.nil || r.nil) return false;
        const int c = l.value.compare(r.value);
        if (op == "<") return c < 0;
        if (op == "<=") return c <= 0;
        if (op == ">") return c > 0;
        return c >= 0;
    }
    if (op == "is_set") return l.found;
    if (op == "is_not_set") return !l.found;
    if (op == "version") return l.found && r.found && version_match(false, l, r);
    if (op == "semver") return l.found && r.found && version_match(true, l, r);
    if (op == "regexp") return l.found && r.found && regexp_match(l, r);
    if (op == "set_contains" || op == "set_contains_all") return l.found && r.found && set_contains(l, r, true);
    if (op == "set_contains_any") return l.found && r.found && set_contains(l, r, false);
    return false;
}

// ---- device attributes ------------------------------------------------------
namespace {
struct UnitInfo { const char* name; uint8_t base; int64_t mult; bool inverse; };
// plugins/shared/structs/units.go: byte, byte-rate, hertz, watt families
const UnitInfo kUnits[] = {
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

const UnitInfo* unit_of(const std::string& u) {
    if (u.empty()) return nullptr;
    for (const auto& x : kUnits) if (u == x.name) return &x;
    return nullptr;
}

bool go_parse_int(const std::string& s, int64_t* out) {   // strconv.ParseInt(s, 10, 64)
    if (s.empty()) return false;
    size_t i = (s[0] == '+' || s[0] == '-') ? 1 : 0;
    if (i == s.size()) return false;
    unsigned __int128 v = 0;
    for (size_t k = i; k < s.size(); k++) {
        if (s[k] < '0' || s[k] > '9') return false;
        v = v * 10 + (unsigned)(s[k] - '0');
        if (v > ((unsigned __int128)1 << 63)) return false;
    }
    const bool neg = s[0] == '-';
    if (!neg && v > (unsigned __int128)INT64_MAX) return false;
    *out = neg ? (int64_t)(0 - (uint64_t)v) : (int64_t)v;
    return true;
}

bool go_parse_float(const std::string& s, double* out) {   // strconv.ParseFloat(s, 64), decimal forms
    if (s.empty()) return false;
    std::string low;
    for (char c : s) low.push_back((char)std::tolower((unsigned char)c));
    const size_t sign = (low[0] == '+' || low[0] == '-') ? 1 : 0;
    const std::string body = low.substr(sign);
    if (body == "inf" || body == "infinity") { *out = low[0] == '-' ? -HUGE_VAL : HUGE_VAL; return true; }
    if (body == "nan" && sign == 0) { *out = std::nan(""); return true; }
    size_t k = sign;
    bool digit = false, dot = false;
    for (; k < low.size(); k++) {
        if (low[k] >= '0' && low[k] <= '9') digit = true;
        else if (low[k] == '.' && !dot) dot = true;
        else break;
    }
    if (!digit) return false;
    if (k < low.size() && low[k] == 'e') {
        k++;
        if (k < low.size() && (low[k] == '+' || low[k] == '-')) k++;
        const size_t e0 = k;
        while (k < low.size() && low[k] >= '0' && low[k] <= '9') k++;
        if (k == e0) return false;
    }
    if (k != low.size()) return false;
    *out = std::strtod(s.c_str(), nullptr);
    return true;
}
}  // namespace

DevAttr parse_dev_attr(const std::string& in) {
    DevAttr a;
    a.kind = DevAttr::kString;
    if (in.empty()) return a;
    std::string unit, numeric = in;
    if (std::isalpha((unsigned char)in.back())) {
        size_t best = 0;   // lengthSortedUnits: the longest matching suffix wins
        for (const auto& u : kUnits) {
            const size_t n = std::strlen(u.name);
            if (n > best && in.size() >= n && in.compare(in.size() - n, n, u.name) == 0) {
                best = n;
                unit = u.name;
            }
        }
        if (!unit.empty()) numeric = strip(in.substr(0, in.size() - unit.size()));
    }
    if (go_parse_int(numeric, &a.i)) { a.kind = DevAttr::kInt; a.unit = unit; return a; }
    if (go_parse_float(numeric, &a.f)) { a.kind = DevAttr::kFloat; a.unit = unit; return a; }
    if (in == "1" || in == "t" || in == "T" || in == "TRUE" || in == "true" || in == "True") {
        a.kind = DevAttr::kBool; a.b = true; return a;
    }
    if (in == "0" || in == "f" || in == "F" || in == "FALSE" || in == "false" || in == "False") {
        a.kind = DevAttr::kBool; a.b = false; return a;
    }
    a.s = in;
    return a;
}

int compare_dev_attr(const DevAttr& a, const DevAttr& b, bool* ok) {
    *ok = false;
    const UnitInfo* ua = unit_of(a.unit);
    const UnitInfo* ub = unit_of(b.unit);
    // Comparable (attribute.go:296-320)
    if (ua || ub) {
        if (!(ua && ub) || ua->base != ub->base) return 0;
    } else if (a.kind == DevAttr::kString && b.kind != DevAttr::kString) {
        return 0;
    } else if (a.kind == DevAttr::kBool && b.kind != DevAttr::kBool) {
        return 0;
    }
    switch (a.kind) {
        case DevAttr::kBool: *ok = true; return a.b == b.b ? 0 : 1;
        case DevAttr::kString: *ok = true; return a.s == b.s ? 0 : (a.s < b.s ? -1 : 1);
        case DevAttr::kInt:
        case DevAttr::kFloat: break;
        default: return 0;   // nullComparator
    }
    if (a.kind == DevAttr::kInt && b.kind == DevAttr::kInt) {   // intComparator on getInt()
        auto scaled = [](const DevAttr& x, const UnitInfo* u) -> int64_t {
            if (!u) return x.i;
            return u->inverse ? x.i / u->mult : (int64_t)((uint64_t)x.i * (uint64_t)u->mult);
        };
        const int64_t x = scaled(a, ua), y = scaled(b, ub);
        *ok = true;
        return x == y ? 0 : (x < y ? -1 : 1);
    }
    if (b.kind != DevAttr::kInt && b.kind != DevAttr::kFloat) return 0;
    // getBigFloat: value x multiplier (1/multiplier for inverse units)
    auto big = [](const DevAttr& x, const UnitInfo* u) -> long double {
        const long double v = x.kind == DevAttr::kInt ? (long double)x.i : (long double)x.f;
        if (!u) return v;
        return u->inverse ? v * (1.0L / (long double)u->mult) : v * (long double)u->mult;
    };
    const long double x = big(a, ua), y = big(b, ub);
    *ok = true;
    return x < y ? -1 : (x > y ? 1 : 0);
}

bool ConstraintEvaluator::check_attr(const std::string& op, const DevAttr& l, bool lf, const DevAttr& r, bool rf) {
    if (op == "distinct_hosts" || op == "distinct_property") return true;
    const bool eq_ops = op == "=" || op == "==" || op == "is";
    const bool ord_ops = op == "<" || op == "<=" || op == ">" || op == ">=";
    if (op == "!=" || op == "not") {
        if (!lf && !rf) return false;
        if (lf != rf) return true;
        bool ok;
        const int v = compare_dev_attr(l, r, &ok);
        return ok && v != 0;
    }
    if (eq_ops || ord_ops) {
        if (!(lf && rf)) return false;
        bool ok;
        const int v = compare_dev_attr(l, r, &ok);
        if (!ok) return false;
        if (eq_ops) return v == 0;
        if (op == "<") return v == -1;
        if (op == "<=") return v != 1;
        if (op == ">") return v == 1;
        return v != -1;
    }
    if (op == "is_set") return lf;
    if (op == "is_not_set") return !lf;
    if (!(lf && rf)) return false;
    if (op == "version" || op == "semver") {   // checkAttributeVersionMatch (feasible.go:896-930)
        Target tl, tr;
        tl.nil = tr.nil = false;
        tl.found = tr.found = true;
        if (l.kind == DevAttr::kString) tl.value = l.s;
        else if (l.kind == DevAttr::kInt) tl.value = std::to_string(l.i);
        else return false;
        if (r.kind != DevAttr::kString) return false;
        tr.value = r.s;
        return version_match(op == "semver", tl, tr);
    }
    if (l.kind != DevAttr::kString || r.kind != DevAttr::kString) return false;
    Target tl, tr;
    tl.nil = tr.nil = false;
    tl.found = tr.found = true;
    tl.value = l.s;
    tr.value = r.s;
    if (op == "regexp") return regexp_match(tl, tr);
    if (op == "set_contains" || op == "set_contains_all") return set_contains(tl, tr, true);
    if (op == "set_contains_any") return set_contains(tl, tr, false);
    return false;
}

bool target_escapes(const std::string& t) {
    return t.rfind("${node.unique.", 0) == 0 || t.rfind("${attr.unique.", 0) == 0 ||
           t.rfind("${meta.unique.", 0) == 0;
}

}  // namespace pe
