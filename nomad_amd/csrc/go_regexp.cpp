// Go 1.16 regexp (RE2 syntax, syntax.Perl flags) for the `regexp` operand.
// See go_regexp.h. Acceptance rules follow Go's regexp/syntax parser
// (src/regexp/syntax/parse.go, Go 1.16.7); the structure here is our own:
// a recursive-descent parser over the pattern bytes producing a small AST of
// code-point sets, assertions and repetitions, a Thompson construction, and a
// state-set simulation. Reference call site: scheduler/feasible.go:931-960.
#include "go_regexp.h"
#include "unicode13.h"

#include <algorithm>
#include <array>
#include <cstring>
#include <map>
#include <vector>

namespace pe {
namespace gore {

namespace {

constexpr uint32_t kMaxRune = 0x10FFFF;
constexpr uint32_t kRuneError = 0xFFFD;
constexpr int kMaxDepth = 1000;     // group / repetition nesting the host stack is allowed to take

using Range = std::pair<uint32_t, uint32_t>;
using RuneSet = std::vector<Range>;   // sorted, merged after normalize()

// utf8.DecodeRuneInString: invalid or truncated sequences decode as
// (RuneError, 1); an empty input as (RuneError, 0).
inline uint32_t decode(const std::string& s, size_t i, size_t* w) {
    const size_t n = s.size() - i;
    const unsigned char* p = reinterpret_cast<const unsigned char*>(s.data()) + i;
    if (n == 0) { *w = 0; return kRuneError; }
    const unsigned b0 = p[0];
    *w = 1;
    if (b0 < 0x80) return b0;
    if (b0 < 0xC2 || b0 > 0xF4) return kRuneError;
    if (b0 < 0xE0) {
        if (n < 2 || (p[1] & 0xC0) != 0x80) return kRuneError;
        *w = 2;
        return ((b0 & 0x1F) << 6) | (p[1] & 0x3F);
    }
    unsigned lo = 0x80, hi = 0xBF;
    if (b0 == 0xE0) lo = 0xA0;
    else if (b0 == 0xED) hi = 0x9F;
    else if (b0 == 0xF0) lo = 0x90;
    else if (b0 == 0xF4) hi = 0x8F;
    if (n < 2 || p[1] < lo || p[1] > hi) return kRuneError;
    if (b0 < 0xF0) {
        if (n < 3 || (p[2] & 0xC0) != 0x80) return kRuneError;
        *w = 3;
        return ((b0 & 0x0F) << 12) | ((p[1] & 0x3F) << 6) | (p[2] & 0x3F);
    }
    if (n < 4 || (p[2] & 0xC0) != 0x80 || (p[3] & 0xC0) != 0x80) return kRuneError;
    *w = 4;
    return ((b0 & 0x07) << 18) | ((p[1] & 0x3F) << 12) | ((p[2] & 0x3F) << 6) | (p[3] & 0x3F);
}

inline bool bad_rune(uint32_t r, size_t w) { return r == kRuneError && w == 1; }

bool valid_utf8(const std::string& s, size_t b, size_t e) {
    std::string t = s.substr(b, e - b);
    for (size_t i = 0; i < t.size();) {
        size_t w;
        const uint32_t r = decode(t, i, &w);
        if (bad_rune(r, w)) return false;
        i += w;
    }
    return true;
}

inline bool ascii_alnum(uint32_t c) {
    return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z');
}
inline bool word_rune(int64_t c) { return c >= 0 && (ascii_alnum((uint32_t)c) || c == '_'); }
inline int hexval(uint32_t c) {
    if (c >= '0' && c <= '9') return (int)(c - '0');
    if (c >= 'a' && c <= 'f') return (int)(c - 'a' + 10);
    if (c >= 'A' && c <= 'F') return (int)(c - 'A' + 10);
    return -1;
}

// ---- code-point sets --------------------------------------------------------

void normalize(RuneSet& s) {
    std::sort(s.begin(), s.end());
    size_t k = 0;
    for (size_t i = 0; i < s.size(); i++) {
        if (k && s[i].first <= s[k - 1].second + 1) s[k - 1].second = std::max(s[k - 1].second, s[i].second);
        else s[k++] = s[i];
    }
    s.resize(k);
}

RuneSet complement(const RuneSet& s) {   // over [0, MaxRune]; s normalized
    RuneSet out;
    uint32_t next = 0;
    for (const auto& r : s) {
        if (r.first > next) out.push_back({next, r.first - 1});
        next = r.second + 1;
    }
    if (next <= kMaxRune) out.push_back({next, kMaxRune});
    return out;
}

bool contains(const RuneSet& s, uint32_t c) {
    size_t lo = 0, hi = s.size();
    while (lo < hi) {
        const size_t m = (lo + hi) / 2;
        if (c < s[m].first) hi = m;
        else if (c > s[m].second) lo = m + 1;
        else return true;
    }
    return false;
}

// Simple-case-folding equivalence classes: the orbits unicode.SimpleFold
// walks (runes with the same CaseFolding.txt C+S image).
const std::vector<std::vector<uint32_t>>& fold_orbits() {
    static const std::vector<std::vector<uint32_t>> orbits = [] {
        std::map<uint32_t, std::vector<uint32_t>> by_image;
        for (uint32_t k = 0; k < ucd13::kNumFold; k++) by_image[ucd13::kFold[k].f].push_back(ucd13::kFold[k].c);
        std::vector<std::vector<uint32_t>> o;
        for (auto& kv : by_image) {
            std::vector<uint32_t> m = kv.second;
            m.push_back(kv.first);
            std::sort(m.begin(), m.end());
            o.push_back(m);
        }
        return o;
    }();
    return orbits;
}

// Close a set under case folding (appendFoldedRange / appendFoldedClass and
// the FoldCategory / FoldScript tables of the reference's Go runtime).
RuneSet fold_closure(const RuneSet& in) {
    RuneSet out = in;
    for (const auto& orbit : fold_orbits()) {
        bool hit = false;
        for (uint32_t c : orbit) hit = hit || contains(in, c);
        if (hit) for (uint32_t c : orbit) out.push_back({c, c});
    }
    normalize(out);
    return out;
}

RuneSet table_set(const ucd13::Range* r, uint32_t n) {
    RuneSet s;
    s.reserve(n);
    for (uint32_t k = 0; k < n; k++) s.push_back({r[k].lo, r[k].hi});
    normalize(s);
    return s;
}

// unicodeTable(name): "Any", then unicode.Categories, then unicode.Scripts.
bool unicode_table(const std::string& name, RuneSet* out) {
    if (name == "Any") { *out = {{0, kMaxRune}}; return true; }
    for (uint32_t k = 0; k < ucd13::kNumCategories; k++)
        if (name == ucd13::kCategories[k].name) { *out = table_set(ucd13::kCategories[k].r, ucd13::kCategories[k].n); return true; }
    for (uint32_t k = 0; k < ucd13::kNumScripts; k++)
        if (name == ucd13::kScripts[k].name) { *out = table_set(ucd13::kScripts[k].r, ucd13::kScripts[k].n); return true; }
    return false;
}

// ASCII groups: [[:name:]] (posixGroup) and \d \s \w (perlGroup).
bool posix_group(const std::string& name, RuneSet* out) {
    static const struct { const char* name; std::vector<Range> r; } kGroups[] = {
        {"alnum", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}},
        {"alpha", {{'A', 'Z'}, {'a', 'z'}}},
        {"ascii", {{0, 0x7F}}},
        {"blank", {{'\t', '\t'}, {' ', ' '}}},
        {"cntrl", {{0, 0x1F}, {0x7F, 0x7F}}},
        {"digit", {{'0', '9'}}},
        {"graph", {{'!', '~'}}},
        {"lower", {{'a', 'z'}}},
        {"print", {{' ', '~'}}},
        {"punct", {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}}},
        {"space", {{'\t', '\r'}, {' ', ' '}}},
        {"upper", {{'A', 'Z'}}},
        {"word", {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}},
        {"xdigit", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}},
    };
    for (const auto& g : kGroups)
        if (name == g.name) { *out = g.r; return true; }
    return false;
}

bool perl_group(char c, RuneSet* out, bool* negated) {
    switch (c) {
        case 'd': case 'D': *out = {{'0', '9'}}; break;
        case 's': case 'S': *out = {{'\t', '\n'}, {'\f', '\r'}, {' ', ' '}}; break;
        case 'w': case 'W': *out = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}; break;
        default: return false;
    }
    *negated = c == 'D' || c == 'S' || c == 'W';
    return true;
}

// ---- AST --------------------------------------------------------------------

enum Kind : uint8_t { kEmpty, kSet, kAssert, kCat, kAlt, kStar, kPlus, kQuest, kRep };
enum Cond : uint8_t { cBeginText = 1, cEndText = 2, cBeginLine = 4, cEndLine = 8, cWordB = 16, cNoWordB = 32 };

struct Node {
    Kind kind = kEmpty;
    uint8_t cond = 0;
    int min = 0, max = 0;
    uint32_t set = 0;
    std::vector<uint32_t> kids;
};

enum Flag { fFold = 1, fOneLine = 2, fDotNL = 4, fNonGreedy = 8 };

class Parser {
public:
    explicit Parser(const std::string& s) : s_(s) {}
    int parse(uint32_t* root) {
        const bool ok = group(fOneLine, true, 0, root);
        return ok ? kOk : (too_deep_ ? kTooLarge : kSyntaxError);
    }
    std::vector<Node> nodes;
    std::vector<RuneSet> sets;

private:
    const std::string& s_;
    size_t i_ = 0;
    mutable bool too_deep_ = false;

    uint32_t add(Node n) { nodes.push_back(std::move(n)); return (uint32_t)nodes.size() - 1; }
    uint32_t set_node(RuneSet s) {
        normalize(s);
        sets.push_back(std::move(s));
        Node n;
        n.kind = kSet;
        n.set = (uint32_t)sets.size() - 1;
        return add(n);
    }
    uint32_t literal(uint32_t c, int flags) {
        RuneSet s{{c, c}};
        if (flags & fFold) s = fold_closure(s);
        return set_node(s);
    }
    uint32_t assert_node(uint8_t cond) { Node n; n.kind = kAssert; n.cond = cond; return add(n); }
    uint32_t wrap(Kind k, uint32_t sub, int mn = 0, int mx = 0) {
        Node n;
        n.kind = k;
        n.min = mn;
        n.max = mx;
        n.kids.push_back(sub);
        return add(n);
    }
    uint32_t seq(Kind k, std::vector<uint32_t>& items) {
        if (items.empty()) return add(Node{});
        if (items.size() == 1) return items[0];
        Node n;
        n.kind = k;
        n.kids = items;
        return add(n);
    }

    // repeatIsValid (parse.go): nested counted repetitions may not multiply
    // past 1000 copies of the innermost expression.
    bool repeat_valid(uint32_t id, int budget, int depth) const {
        if (depth > kMaxDepth) { too_deep_ = true; return false; }
        const Node& n = nodes[id];
        if (n.kind == kRep) {
            int m = n.max;
            if (m == 0) return true;
            if (m < 0) m = n.min;
            if (m > budget) return false;
            if (m > 0) budget /= m;
        }
        for (uint32_t k : n.kids) if (!repeat_valid(k, budget, depth + 1)) return false;
        return true;
    }

    // parseInt: decimal without leading zeros; values >= 1e8 become -1.
    bool parse_int(size_t* p, int* v) const {
        size_t j = *p;
        if (j >= s_.size() || s_[j] < '0' || s_[j] > '9') return false;
        if (j + 1 < s_.size() && s_[j] == '0' && s_[j + 1] >= '0' && s_[j + 1] <= '9') return false;
        long long acc = 0;
        bool big = false;
        while (j < s_.size() && s_[j] >= '0' && s_[j] <= '9') {
            if (!big) {
                if (acc >= 100000000) big = true;
                else acc = acc * 10 + (s_[j] - '0');
            }
            j++;
        }
        *v = big ? -1 : (int)acc;
        *p = j;
        return true;
    }

    // parseRepeat: {n}, {n,}, {n,m}; anything else leaves '{' a literal.
    bool repeat_spec(int* mn, int* mx, size_t* after) const {
        size_t j = i_ + 1;
        if (!parse_int(&j, mn)) return false;
        if (j >= s_.size()) return false;
        if (s_[j] != ',') {
            *mx = *mn;
        } else {
            j++;
            if (j >= s_.size()) return false;
            if (s_[j] == '}') *mx = -1;
            else {
                if (!parse_int(&j, mx)) return false;
                if (*mx < 0) *mn = -1;
            }
        }
        if (j >= s_.size() || s_[j] != '}') return false;
        *after = j + 1;
        return true;
    }

    // parseEscape: one escaped rune at i_ (pointing at the backslash).
    bool escape_rune(uint32_t* out) {
        size_t j = i_ + 1;
        if (j >= s_.size()) return false;   // trailing backslash
        size_t w;
        uint32_t c = decode(s_, j, &w);
        if (bad_rune(c, w)) return false;
        j += w;
        if (c < 0x80 && !ascii_alnum(c)) { *out = c; i_ = j; return true; }
        auto octal = [&](size_t k) { return k < s_.size() && s_[k] >= '0' && s_[k] <= '7'; };
        switch (c) {
            case '1': case '2': case '3': case '4': case '5': case '6': case '7':
                if (!octal(j)) return false;   // a backreference: unsupported
                [[fallthrough]];
            case '0': {
                uint32_t r = c - '0';
                for (int k = 1; k < 3 && octal(j); k++) r = r * 8 + (uint32_t)(s_[j++] - '0');
                *out = r;
                i_ = j;
                return true;
            }
            case 'x': {
                if (j >= s_.size()) return false;
                c = decode(s_, j, &w);
                if (bad_rune(c, w)) return false;
                j += w;
                if (c == '{') {
                    int nhex = 0;
                    uint32_t r = 0;
                    for (;;) {
                        if (j >= s_.size()) return false;
                        c = decode(s_, j, &w);
                        if (bad_rune(c, w)) return false;
                        j += w;
                        if (c == '}') break;
                        const int v = hexval(c);
                        if (v < 0) return false;
                        r = r * 16 + (uint32_t)v;
                        if (r > kMaxRune) return false;
                        nhex++;
                    }
                    if (nhex == 0) return false;
                    *out = r;
                    i_ = j;
                    return true;
                }
                const int x = hexval(c);
                c = decode(s_, j, &w);   // at the end: (RuneError, 0), not a hex digit
                if (bad_rune(c, w)) return false;
                j += w;
                const int y = hexval(c);
                if (x < 0 || y < 0) return false;
                *out = (uint32_t)(x * 16 + y);
                i_ = j;
                return true;
            }
            case 'a': *out = 7; break;
            case 'f': *out = 12; break;
            case 'n': *out = 10; break;
            case 'r': *out = 13; break;
            case 't': *out = 9; break;
            case 'v': *out = 11; break;
            default: return false;
        }
        i_ = j;
        return true;
    }

    // parseUnicodeClass at i_ (\p or \P). *hit = false when i_ is not one.
    bool unicode_class(int flags, RuneSet* out, bool* hit) {
        *hit = false;
        if (i_ + 1 >= s_.size() || s_[i_] != '\\' || (s_[i_ + 1] != 'p' && s_[i_ + 1] != 'P')) return true;
        *hit = true;
        bool neg = s_[i_ + 1] == 'P';
        size_t j = i_ + 2, w;
        const uint32_t c = decode(s_, j, &w);
        if (bad_rune(c, w)) return false;
        std::string name;
        if (c != '{') {
            name = s_.substr(j, w);
            j += w;
        } else {
            const size_t end = s_.find('}', i_);
            if (end == std::string::npos) return false;
            name = s_.substr(i_ + 3, end - (i_ + 3));
            if (!valid_utf8(name, 0, name.size())) return false;
            j = end + 1;
        }
        if (!name.empty() && name[0] == '^') { neg = !neg; name = name.substr(1); }
        RuneSet t;
        if (!unicode_table(name, &t)) return false;
        if (flags & fFold) t = fold_closure(t);
        *out = neg ? complement(t) : t;
        i_ = j;
        return true;
    }

    // A \d \D \s \S \w \W escape at i_ as a set (folded, then negated).
    bool perl_class(int flags, RuneSet* out) {
        if (i_ + 1 >= s_.size() || s_[i_] != '\\') return false;
        bool neg;
        RuneSet g;
        if (!perl_group(s_[i_ + 1], &g, &neg)) return false;
        if (flags & fFold) g = fold_closure(g);
        *out = neg ? complement(g) : g;
        i_ += 2;
        return true;
    }

    // parseClass: i_ at '['.
    bool char_class(int flags, uint32_t* out) {
        const size_t n = s_.size();
        i_++;
        bool neg = false;
        if (i_ < n && s_[i_] == '^') { neg = true; i_++; }
        RuneSet cls;
        bool first = true;
        while (i_ >= n || s_[i_] != ']' || first) {
            first = false;
            if (n - std::min(n, i_) > 2 && s_[i_] == '[' && s_[i_ + 1] == ':') {
                const size_t e = s_.find(":]", i_ + 2);
                if (e != std::string::npos) {
                    std::string name = s_.substr(i_ + 2, e - (i_ + 2));
                    bool gneg = false;
                    if (!name.empty() && name[0] == '^') { gneg = true; name = name.substr(1); }
                    RuneSet g;
                    if (!posix_group(name, &g)) return false;
                    if (flags & fFold) g = fold_closure(g);
                    if (gneg) g = complement(g);
                    cls.insert(cls.end(), g.begin(), g.end());
                    i_ = e + 2;
                    continue;
                }
            }
            RuneSet g;
            bool hit;
            if (!unicode_class(flags, &g, &hit)) return false;
            if (!hit && perl_class(flags, &g)) hit = true;
            if (hit) { cls.insert(cls.end(), g.begin(), g.end()); continue; }
            uint32_t lo, hi;
            if (!class_char(&lo)) return false;
            hi = lo;
            if (i_ + 1 < n && s_[i_] == '-' && s_[i_ + 1] != ']') {
                i_++;
                if (!class_char(&hi)) return false;
                if (hi < lo) return false;
            }
            RuneSet r{{lo, hi}};
            if (flags & fFold) r = fold_closure(r);
            cls.insert(cls.end(), r.begin(), r.end());
        }
        i_++;   // ']'
        normalize(cls);
        if (neg) cls = complement(cls);
        *out = set_node(cls);
        return true;
    }

    bool class_char(uint32_t* out) {
        if (i_ >= s_.size()) return false;   // missing closing ]
        if (s_[i_] == '\\') return escape_rune(out);
        size_t w;
        const uint32_t c = decode(s_, i_, &w);
        if (bad_rune(c, w)) return false;
        i_ += w;
        *out = c;
        return true;
    }

    // "(?" at i_: named capture, flag group (?flags:re) or flag change (?flags).
    bool perl_paren(int* flags, std::vector<uint32_t>& items, int depth) {
        const size_t n = s_.size();
        if (n - i_ > 4 && s_[i_ + 2] == 'P' && s_[i_ + 3] == '<') {
            const size_t end = s_.find('>', i_);
            if (end == std::string::npos) return false;
            if (!valid_utf8(s_, i_ + 4, end)) return false;
            if (end == i_ + 4) return false;
            for (size_t k = i_ + 4; k < end; k++)
                if (!(ascii_alnum((unsigned char)s_[k]) || s_[k] == '_')) return false;
            i_ = end + 1;
            uint32_t g;
            if (!group(*flags, false, depth + 1, &g)) return false;
            items.push_back(g);
            return true;
        }
        size_t j = i_ + 2;
        int f = *flags;
        bool negate = false, saw = false;
        while (j < n) {
            size_t w;
            const uint32_t c = decode(s_, j, &w);
            if (bad_rune(c, w)) return false;
            j += w;
            switch (c) {
                case 'i': f |= fFold; saw = true; break;
                case 'm': f &= ~fOneLine; saw = true; break;
                case 's': f |= fDotNL; saw = true; break;
                case 'U': f |= fNonGreedy; saw = true; break;
                case '-':
                    if (negate) return false;
                    negate = true;
                    f = ~f;   // set bits now clear them once inverted back
                    saw = false;
                    break;
                case ':': case ')':
                    if (negate) {
                        if (!saw) return false;
                        f = ~f;
                    }
                    i_ = j;
                    if (c == ')') { *flags = f; return true; }
                    {
                        uint32_t g;
                        if (!group(f, false, depth + 1, &g)) return false;
                        items.push_back(g);
                    }
                    return true;
                default:
                    return false;   // lookaround, (?<name>, (?P=name), unknown flags
            }
        }
        return false;
    }

    // The whole pattern (top) or the body of one group after its '('. Flag
    // changes made inside last until the group closes.
    bool group(int flags, bool top, int depth, uint32_t* out) {
        if (depth > kMaxDepth) { too_deep_ = true; return false; }
        const size_t n = s_.size();
        std::vector<uint32_t> alts, items;
        bool after_repeat = false;
        for (;;) {
            if (i_ >= n) {
                if (!top) return false;   // missing closing )
                break;
            }
            const char c = s_[i_];
            if (c == ')') {
                if (top) return false;    // unexpected )
                i_++;
                break;
            }
            if (c == '|') {
                alts.push_back(seq(kCat, items));
                items.clear();
                i_++;
                after_repeat = false;
                continue;
            }
            if (c == '*' || c == '+' || c == '?') {
                i_++;
                if (i_ < n && s_[i_] == '?') i_++;   // non-greedy
                if (after_repeat || items.empty()) return false;   // a** / missing argument
                items.back() = wrap(c == '*' ? kStar : c == '+' ? kPlus : kQuest, items.back());
                after_repeat = true;
                continue;
            }
            if (c == '{') {
                int mn, mx;
                size_t after;
                if (repeat_spec(&mn, &mx, &after)) {
                    if (mn < 0 || mn > 1000 || mx > 1000 || (mx >= 0 && mn > mx)) return false;
                    i_ = after;
                    if (i_ < n && s_[i_] == '?') i_++;
                    if (after_repeat || items.empty()) return false;
                    const uint32_t r = wrap(kRep, items.back(), mn, mx);
                    if ((mn >= 2 || mx >= 2) && !repeat_valid(r, 1000, 0)) return false;
                    items.back() = r;
                    after_repeat = true;
                    continue;
                }
                items.push_back(literal('{', flags));
                i_++;
                after_repeat = false;
                continue;
            }
            after_repeat = false;
            switch (c) {
                case '(':
                    if (i_ + 1 < n && s_[i_ + 1] == '?') {
                        if (!perl_paren(&flags, items, depth)) return false;
                    } else {
                        i_++;
                        uint32_t g;
                        if (!group(flags, false, depth + 1, &g)) return false;
                        items.push_back(g);
                    }
                    break;
                case '^':
                    items.push_back(assert_node((flags & fOneLine) ? cBeginText : cBeginLine));
                    i_++;
                    break;
                case '$':
                    items.push_back(assert_node((flags & fOneLine) ? cEndText : cEndLine));
                    i_++;
                    break;
                case '.':
                    items.push_back(set_node((flags & fDotNL) ? RuneSet{{0, kMaxRune}}
                                                              : RuneSet{{0, '\n' - 1}, {'\n' + 1, kMaxRune}}));
                    i_++;
                    break;
                case '[': {
                    uint32_t g;
                    if (!char_class(flags, &g)) return false;
                    items.push_back(g);
                    break;
                }
                case '\\': {
                    if (i_ + 1 < n) {
                        const char e = s_[i_ + 1];
                        if (e == 'A' || e == 'z' || e == 'b' || e == 'B') {
                            items.push_back(assert_node(e == 'A' ? cBeginText : e == 'z' ? cEndText
                                                        : e == 'b' ? cWordB : cNoWordB));
                            i_ += 2;
                            break;
                        }
                        if (e == 'C') return false;   // any byte: unsupported
                        if (e == 'Q') {               // \Q...\E: literal text
                            const size_t end = s_.find("\\E", i_ + 2);
                            const size_t stop = end == std::string::npos ? n : end;
                            size_t j = i_ + 2;
                            while (j < stop) {
                                size_t w;
                                const uint32_t r = decode(s_, j, &w);
                                if (bad_rune(r, w)) return false;
                                items.push_back(literal(r, flags));
                                j += w;
                            }
                            i_ = end == std::string::npos ? n : end + 2;
                            break;
                        }
                    }
                    RuneSet g;
                    bool hit;
                    if (!unicode_class(flags, &g, &hit)) return false;
                    if (hit || perl_class(flags, &g)) { items.push_back(set_node(g)); break; }
                    uint32_t r;
                    if (!escape_rune(&r)) return false;
                    items.push_back(literal(r, flags));
                    break;
                }
                default: {
                    size_t w;
                    const uint32_t r = decode(s_, i_, &w);
                    if (bad_rune(r, w)) return false;
                    items.push_back(literal(r, flags));
                    i_ += w;
                }
            }
        }
        alts.push_back(seq(kCat, items));
        *out = seq(kAlt, alts);
        return true;
    }
};

}  // namespace

// ---- program ------------------------------------------------------------------

enum Op : uint8_t { iRune, iSplit, iNop, iEmpty, iMatch };

struct Inst {
    Op op;
    uint8_t cond;
    uint32_t out, out1;
    uint32_t set;
};

struct Prog {
    std::vector<Inst> inst;
    std::vector<RuneSet> sets;
    std::vector<std::array<uint64_t, 2>> ascii;   // per set: membership of runes < 128
    uint32_t start = 0;
};

namespace {

struct Frag {
    uint32_t start;
    std::vector<uint32_t> holes;   // inst * 2 + (0: out, 1: out1)
};

class Compiler {
public:
    Compiler(const std::vector<Node>& nodes, Prog* p) : nodes_(nodes), p_(p) {}
    bool overflow = false;

    Frag emit(uint32_t id, int depth) {
        if (overflow || depth > 4 * kMaxDepth) { overflow = true; return nop(); }
        const Node& n = nodes_[id];
        switch (n.kind) {
            case kEmpty: return nop();
            case kSet: {
                const uint32_t k = inst(iRune, 0, n.set);
                return Frag{k, {k * 2}};
            }
            case kAssert: {
                const uint32_t k = inst(iEmpty, n.cond, 0);
                return Frag{k, {k * 2}};
            }
            case kCat: {
                Frag f = emit(n.kids[0], depth + 1);
                for (size_t k = 1; k < n.kids.size(); k++) f = cat(f, emit(n.kids[k], depth + 1));
                return f;
            }
            case kAlt: {
                Frag f = emit(n.kids.back(), depth + 1);
                for (size_t k = n.kids.size() - 1; k-- > 0;) f = alt(emit(n.kids[k], depth + 1), f);
                return f;
            }
            case kStar: return star(emit(n.kids[0], depth + 1));
            case kPlus: return plus(emit(n.kids[0], depth + 1));
            case kQuest: return quest(emit(n.kids[0], depth + 1));
            case kRep: {
                // x{n,m}: n copies, then m-n nested optional copies; x{n,}: n-1 copies and x+.
                const uint32_t x = n.kids[0];
                if (n.max < 0) {
                    if (n.min == 0) return star(emit(x, depth + 1));
                    Frag f = nop();
                    for (int k = 0; k + 1 < n.min && !overflow; k++) f = cat(f, emit(x, depth + 1));
                    return cat(f, plus(emit(x, depth + 1)));
                }
                Frag f = nop();
                for (int k = 0; k < n.min && !overflow; k++) f = cat(f, emit(x, depth + 1));
                if (n.max > n.min) {
                    Frag tail = quest(emit(x, depth + 1));
                    for (int k = n.min + 1; k < n.max && !overflow; k++) tail = quest(cat(emit(x, depth + 1), tail));
                    f = cat(f, tail);
                }
                return f;
            }
        }
        return nop();
    }

    void patch(const std::vector<uint32_t>& holes, uint32_t to) {
        for (uint32_t h : holes) (h & 1 ? p_->inst[h >> 1].out1 : p_->inst[h >> 1].out) = to;
    }
    uint32_t inst(Op op, uint8_t cond, uint32_t set) {
        if (p_->inst.size() >= kMaxInst) { overflow = true; return 0; }
        p_->inst.push_back(Inst{op, cond, 0, 0, set});
        return (uint32_t)p_->inst.size() - 1;
    }

private:
    const std::vector<Node>& nodes_;
    Prog* p_;

    Frag nop() {
        const uint32_t k = inst(iNop, 0, 0);
        return Frag{k, {k * 2}};
    }
    Frag cat(Frag a, const Frag& b) {
        patch(a.holes, b.start);
        return Frag{a.start, b.holes};
    }
    Frag alt(const Frag& a, const Frag& b) {
        const uint32_t k = inst(iSplit, 0, 0);
        if (overflow) return a;
        p_->inst[k].out = a.start;
        p_->inst[k].out1 = b.start;
        Frag f{k, a.holes};
        f.holes.insert(f.holes.end(), b.holes.begin(), b.holes.end());
        return f;
    }
    Frag star(const Frag& a) {
        const uint32_t k = inst(iSplit, 0, 0);
        if (overflow) return a;
        p_->inst[k].out = a.start;
        patch(a.holes, k);
        return Frag{k, {k * 2 + 1}};
    }
    Frag plus(const Frag& a) {
        const uint32_t k = inst(iSplit, 0, 0);
        if (overflow) return a;
        p_->inst[k].out = a.start;
        patch(a.holes, k);
        return Frag{a.start, {k * 2 + 1}};
    }
    Frag quest(const Frag& a) {
        const uint32_t k = inst(iSplit, 0, 0);
        if (overflow) return a;
        p_->inst[k].out = a.start;
        Frag f{k, a.holes};
        f.holes.push_back(k * 2 + 1);
        return f;
    }
};

// Sparse set of instruction indices (Briggs-Torczon), O(1) clear.
struct StateSet {
    std::vector<uint32_t> dense, sparse;
    size_t n = 0;
    explicit StateSet(size_t cap) : dense(cap), sparse(cap) {}
    bool has(uint32_t k) const { return sparse[k] < n && dense[sparse[k]] == k; }
    void insert(uint32_t k) { sparse[k] = (uint32_t)n; dense[n++] = k; }
    void clear() { n = 0; }
};

inline bool in_set(const Prog& p, uint32_t set, uint32_t r) {
    if (r < 128) return (p.ascii[set][r >> 6] >> (r & 63)) & 1;
    return contains(p.sets[set], r);
}

}  // namespace

std::shared_ptr<const Prog> compile(const std::string& expr, int* status) {
    Parser ps(expr);
    uint32_t root;
    *status = ps.parse(&root);
    if (*status != kOk) return nullptr;
    auto p = std::make_shared<Prog>();
    p->sets = std::move(ps.sets);
    Compiler cc(ps.nodes, p.get());
    Frag f = cc.emit(root, 0);
    const uint32_t m = cc.inst(iMatch, 0, 0);
    if (cc.overflow) { *status = kTooLarge; return nullptr; }
    cc.patch(f.holes, m);
    p->start = f.start;
    p->ascii.resize(p->sets.size());
    for (size_t k = 0; k < p->sets.size(); k++) {
        p->ascii[k] = {0, 0};
        for (uint32_t r = 0; r < 128; r++)
            if (contains(p->sets[k], r)) p->ascii[k][r >> 6] |= 1ull << (r & 63);
    }
    return p;
}

bool match(const Prog& p, const std::string& text) {
    const size_t ni = p.inst.size();
    StateSet cur(ni);
    std::vector<uint32_t> pending, stack;
    int64_t prev = -1;   // rune before the position, -1 at the start
    for (size_t i = 0;;) {
        size_t w = 0;
        const int64_t next = i < text.size() ? (int64_t)decode(text, i, &w) : -1;
        uint8_t ctx = 0;
        if (prev < 0) ctx |= cBeginText | cBeginLine;
        else if (prev == '\n') ctx |= cBeginLine;
        if (next < 0) ctx |= cEndText | cEndLine;
        else if (next == '\n') ctx |= cEndLine;
        ctx |= word_rune(prev) != word_rune(next) ? cWordB : cNoWordB;
        // Threads carried over from the previous rune, then a new thread
        // starting here (unanchored search); epsilon closure under ctx.
        cur.clear();
        stack.assign(pending.rbegin(), pending.rend());
        stack.push_back(p.start);
        while (!stack.empty()) {
            const uint32_t k = stack.back();
            stack.pop_back();
            if (cur.has(k)) continue;
            cur.insert(k);
            const Inst& in = p.inst[k];
            switch (in.op) {
                case iMatch: return true;
                case iSplit: stack.push_back(in.out1); stack.push_back(in.out); break;
                case iNop: stack.push_back(in.out); break;
                case iEmpty: if ((in.cond & ~ctx) == 0) stack.push_back(in.out); break;
                case iRune: break;
            }
        }
        if (next < 0) return false;
        pending.clear();
        for (size_t d = 0; d < cur.n; d++) {
            const Inst& in = p.inst[cur.dense[d]];
            if (in.op == iRune && in_set(p, in.set, (uint32_t)next)) pending.push_back(in.out);
        }
        prev = next;
        i += w;
    }
}

bool match_string(const std::string& expr, const std::string& text) {
    int st;
    auto p = compile(expr, &st);
    return p && match(*p, text);
}

}  // namespace gore
}  // namespace pe
