// ORACLE — test infrastructure only (never linked into the product).
//
// Restatement of Go 1.16.7's regexp package as the reference's
// checkRegexpMatch uses it (scheduler/feasible.go:931-960: regexp.Compile,
// error => false, then MatchString). Go's stdlib is a third-party dependency
// absent from /root/reference; this follows its published algorithm:
//   * parse: src/regexp/syntax/parse.go with syntax.Perl flags (ClassNL |
//     OneLine | PerlX | UnicodeGroups): the operator stack with "(" and "|"
//     pseudo-operators, concat / alternate / swapVerticalBar /
//     parseRightParen, lastRepeat (a** is an error), repeat + repeatIsValid
//     (1000), parseRepeat / parseInt, parsePerlFlags (named captures, flag
//     groups), parseClass / parseNamedClass / parseUnicodeClass /
//     parsePerlClassEscape / parseEscape, nextRune / checkUTF8;
//   * classes as Go builds them: items folded with unicode.SimpleFold orbits
//     before negation (appendFoldedRange, appendFoldedClass, FoldCategory /
//     FoldScript), the class negated last;
//   * MatchString as a set semantics: some rune-aligned substring is in the
//     language, with EmptyOpContext assertions (^ $ \A \z \b \B, (?m)).
// Written independently of the product (nomad_amd/csrc/go_regexp.cpp): a
// stack parser here vs recursive descent there; membership by orbit test here
// vs materialised folded sets there; position-set evaluation over the tree
// here vs a Thompson NFA there. Shared input: the Unicode 13.0.0 data header
// (generated data, checked against Python's unicodedata in tests/test_re2.py).
#pragma once
#include <algorithm>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "../nomad_amd/csrc/unicode13.h"

namespace orare {

enum Op {
    NoMatch, EmptyMatch, Literal, CharClass, AnyCharNotNL, AnyChar, BeginLine, EndLine, BeginText, EndText,
    WordBoundary, NoWordBoundary, Capture, Star, Plus, Quest, Repeat, Concat, Alternate,
    Pseudo = 128, LeftParen, VerticalBar
};

enum Flags { FoldCase = 1, OneLine = 2, DotNL = 4, NonGreedy = 8, ClassNL = 16, PerlX = 32, UnicodeGroups = 64 };

struct ClassItem {
    std::vector<std::pair<uint32_t, uint32_t>> base;
    bool fold = false, neg = false;
};

struct Re {
    int op = NoMatch;
    int flags = 0;
    uint32_t rune = 0;              // Literal
    std::vector<ClassItem> items;   // CharClass
    bool negated = false;           // CharClass: [^...]
    int min = 0, max = 0;
    int cap = 0;
    std::vector<int> sub;
};

inline bool in_ranges(const std::vector<std::pair<uint32_t, uint32_t>>& r, uint32_t c) {
    for (auto& x : r) if (c >= x.first && c <= x.second) return true;
    return false;
}

// unicode.SimpleFold orbit of c: all runes whose simple case fold equals c's.
inline uint32_t scf(uint32_t c) {
    size_t lo = 0, hi = ucd13::kNumFold;
    while (lo < hi) {
        size_t m = (lo + hi) / 2;
        if (ucd13::kFold[m].c == c) return ucd13::kFold[m].f;
        if (ucd13::kFold[m].c < c) lo = m + 1; else hi = m;
    }
    return c;
}
inline std::vector<uint32_t> orbit(uint32_t c) {
    static const std::map<uint32_t, std::vector<uint32_t>> members = [] {
        std::map<uint32_t, std::vector<uint32_t>> m;
        for (uint32_t k = 0; k < ucd13::kNumFold; k++) m[ucd13::kFold[k].f].push_back(ucd13::kFold[k].c);
        return m;
    }();
    const uint32_t f = scf(c);
    std::vector<uint32_t> o{f};
    auto it = members.find(f);
    if (it != members.end()) o.insert(o.end(), it->second.begin(), it->second.end());
    return o;
}

inline bool item_has(const ClassItem& it, uint32_t c) {
    bool in = false;
    if (!it.fold) in = in_ranges(it.base, c);
    else for (uint32_t d : orbit(c)) if (in_ranges(it.base, d)) { in = true; break; }
    return in != it.neg;
}

// utf8.DecodeRuneInString
inline uint32_t decode_rune(const std::string& s, size_t i, size_t* size) {
    const unsigned char* p = (const unsigned char*)s.data() + i;
    const size_t n = s.size() - i;
    if (n == 0) { *size = 0; return 0xFFFD; }
    *size = 1;
    if (p[0] < 0x80) return p[0];
    int need;
    uint32_t r;
    unsigned lo = 0x80, hi = 0xBF;
    if (p[0] >= 0xC2 && p[0] <= 0xDF) { need = 1; r = p[0] & 0x1F; }
    else if (p[0] >= 0xE0 && p[0] <= 0xEF) {
        need = 2; r = p[0] & 0x0F;
        if (p[0] == 0xE0) lo = 0xA0;
        if (p[0] == 0xED) hi = 0x9F;
    } else if (p[0] >= 0xF0 && p[0] <= 0xF4) {
        need = 3; r = p[0] & 0x07;
        if (p[0] == 0xF0) lo = 0x90;
        if (p[0] == 0xF4) hi = 0x8F;
    } else return 0xFFFD;
    if (n < (size_t)need + 1) return 0xFFFD;
    for (int k = 1; k <= need; k++) {
        const unsigned b = p[k];
        const unsigned l = k == 1 ? lo : 0x80, h = k == 1 ? hi : 0xBF;
        if (b < l || b > h) return 0xFFFD;
        r = (r << 6) | (b & 0x3F);
    }
    *size = need + 1;
    return r;
}

struct SyntaxError {};

class GoParser {
public:
    std::vector<Re> pool;
    std::vector<int> stack;
    int flags = ClassNL | OneLine | PerlX | UnicodeGroups;   // syntax.Perl
    int numCap = 0;
    std::string whole;

    int newRe(int op) { Re r; r.op = op; r.flags = flags; pool.push_back(r); return (int)pool.size() - 1; }
    Re& at(int k) { return pool[k]; }
    int push(int k) { stack.push_back(k); return k; }
    int op(int o) { return push(newRe(o)); }
    void literal(uint32_t r) {
        const int k = newRe(Literal);
        at(k).rune = r;
        push(k);
    }

    // nextRune
    uint32_t nextRune(const std::string& t, size_t& i) {
        size_t sz;
        const uint32_t c = decode_rune(t, i, &sz);
        if (c == 0xFFFD && sz == 1) throw SyntaxError();
        i += sz;
        return c;
    }
    void checkUTF8(const std::string& t) {
        size_t i = 0;
        while (i < t.size()) nextRune(t, i);
    }

    void concat() {
        size_t i = stack.size();
        while (i > 0 && at(stack[i - 1]).op < Pseudo) i--;
        std::vector<int> subs(stack.begin() + i, stack.end());
        stack.resize(i);
        if (subs.empty()) { op(EmptyMatch); return; }
        if (subs.size() == 1) { push(subs[0]); return; }
        const int k = newRe(Concat);
        at(k).sub = subs;
        push(k);
    }
    void alternate() {
        size_t i = stack.size();
        while (i > 0 && at(stack[i - 1]).op < Pseudo) i--;
        std::vector<int> subs(stack.begin() + i, stack.end());
        stack.resize(i);
        if (subs.empty()) { op(NoMatch); return; }
        if (subs.size() == 1) { push(subs[0]); return; }
        const int k = newRe(Alternate);
        at(k).sub = subs;
        push(k);
    }
    bool swapVerticalBar() {
        const size_t n = stack.size();
        if (n >= 2 && at(stack[n - 2]).op == VerticalBar) {
            std::swap(stack[n - 2], stack[n - 1]);
            return true;
        }
        return false;
    }
    void parseVerticalBar() {
        concat();
        if (!swapVerticalBar()) op(VerticalBar);
    }
    void parseRightParen() {
        concat();
        if (swapVerticalBar()) stack.pop_back();
        alternate();
        const size_t n = stack.size();
        if (n < 2) throw SyntaxError();   // unexpected )
        const int re1 = stack[n - 1], re2 = stack[n - 2];
        stack.resize(n - 2);
        if (at(re2).op != LeftParen) throw SyntaxError();
        flags = at(re2).flags;
        if (at(re2).cap == 0) push(re1);
        else {
            at(re2).op = Capture;
            at(re2).sub = {re1};
            push(re2);
        }
    }

    static bool repeatIsValid(const std::vector<Re>& pool, int k, int n) {
        const Re& re = pool[k];
        if (re.op == Repeat) {
            int m = re.max;
            if (m == 0) return true;
            if (m < 0) m = re.min;
            if (m > n) return false;
            if (m > 0) n /= m;
        }
        for (int s : re.sub) if (!repeatIsValid(pool, s, n)) return false;
        return true;
    }

    // repeat(op, min, max, before, after, lastRepeat): returns the new position.
    size_t repeat(int o, int mn, int mx, size_t after, bool lastRepeat, const std::string& t) {
        int fl = flags;
        if (after < t.size() && t[after] == '?') { after++; fl ^= NonGreedy; }
        if (lastRepeat) throw SyntaxError();    // invalid nested repetition operator
        if (stack.empty()) throw SyntaxError();  // missing argument to repetition operator
        const int sub = stack.back();
        if (at(sub).op >= Pseudo) throw SyntaxError();
        const int k = newRe(o);
        at(k).min = mn;
        at(k).max = mx;
        at(k).flags = fl;
        at(k).sub = {sub};
        stack.back() = k;
        if (o == Repeat && (mn >= 2 || mx >= 2) && !repeatIsValid(pool, k, 1000)) throw SyntaxError();
        return after;
    }

    // parseInt: no leading zeros; >= 1e8 overflows to -1.
    static bool parseInt(const std::string& t, size_t& i, int& n) {
        if (i >= t.size() || t[i] < '0' || t[i] > '9') return false;
        if (t.size() - i >= 2 && t[i] == '0' && t[i + 1] >= '0' && t[i + 1] <= '9') return false;
        const size_t b = i;
        while (i < t.size() && t[i] >= '0' && t[i] <= '9') i++;
        n = 0;
        for (size_t k = b; k < i; k++) {
            if (n >= 100000000) { n = -1; break; }
            n = n * 10 + (t[k] - '0');
        }
        return true;
    }
    static bool parseRepeat(const std::string& t, size_t i, int& mn, int& mx, size_t& rest) {
        if (i >= t.size() || t[i] != '{') return false;
        i++;
        if (!parseInt(t, i, mn)) return false;
        if (i >= t.size()) return false;
        if (t[i] != ',') mx = mn;
        else {
            i++;
            if (i >= t.size()) return false;
            if (t[i] == '}') mx = -1;
            else {
                if (!parseInt(t, i, mx)) return false;
                if (mx < 0) mn = -1;
            }
        }
        if (i >= t.size() || t[i] != '}') return false;
        rest = i + 1;
        return true;
    }

    static bool isalnum_(uint32_t c) {
        return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z');
    }
    static int unhex(uint32_t c) {
        if ('0' <= c && c <= '9') return c - '0';
        if ('a' <= c && c <= 'f') return c - 'a' + 10;
        if ('A' <= c && c <= 'F') return c - 'A' + 10;
        return -1;
    }

    // parseEscape: t[i] is the backslash.
    uint32_t parseEscape(const std::string& t, size_t& i) {
        size_t j = i + 1;
        if (j >= t.size()) throw SyntaxError();   // trailing backslash
        uint32_t c = nextRune(t, j);
        if (c < 0x80 && !isalnum_(c)) { i = j; return c; }
        if (c >= '1' && c <= '7') {
            if (j >= t.size() || t[j] < '0' || t[j] > '7') throw SyntaxError();
        }
        if (c >= '0' && c <= '7') {
            uint32_t r = c - '0';
            for (int k = 1; k < 3; k++) {
                if (j >= t.size() || t[j] < '0' || t[j] > '7') break;
                r = r * 8 + (t[j] - '0');
                j++;
            }
            i = j;
            return r;
        }
        if (c == 'x') {
            if (j >= t.size()) throw SyntaxError();
            c = nextRune(t, j);
            if (c == '{') {
                int nhex = 0;
                uint32_t r = 0;
                for (;;) {
                    if (j >= t.size()) throw SyntaxError();
                    c = nextRune(t, j);
                    if (c == '}') break;
                    const int v = unhex(c);
                    if (v < 0) throw SyntaxError();
                    r = r * 16 + v;
                    if (r > 0x10FFFF) throw SyntaxError();
                    nhex++;
                }
                if (nhex == 0) throw SyntaxError();
                i = j;
                return r;
            }
            const int x = unhex(c);
            uint32_t c2 = 0xFFFD;
            if (j < t.size()) c2 = nextRune(t, j);
            const int y = unhex(c2);
            if (x < 0 || y < 0) throw SyntaxError();
            i = j;
            return x * 16 + y;
        }
        static const char* kC = "a\af\fn\nr\rt\tv\v";
        for (const char* p = kC; *p; p += 2)
            if (c == (uint32_t)p[0]) { i = j; return (uint32_t)p[1]; }
        throw SyntaxError();   // invalid escape
    }

    static std::vector<std::pair<uint32_t, uint32_t>> perlGroup(char c) {
        if (c == 'd' || c == 'D') return {{'0', '9'}};
        if (c == 's' || c == 'S') return {{'\t', '\n'}, {'\f', '\r'}, {' ', ' '}};
        if (c == 'w' || c == 'W') return {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}};
        return {};
    }
    static bool posixGroup(const std::string& name, std::vector<std::pair<uint32_t, uint32_t>>& r) {
        static const std::map<std::string, std::vector<std::pair<uint32_t, uint32_t>>> g = {
            {"alnum", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}}, {"alpha", {{'A', 'Z'}, {'a', 'z'}}},
            {"ascii", {{0, 0x7F}}}, {"blank", {{'\t', '\t'}, {' ', ' '}}},
            {"cntrl", {{0, 0x1F}, {0x7F, 0x7F}}}, {"digit", {{'0', '9'}}}, {"graph", {{'!', '~'}}},
            {"lower", {{'a', 'z'}}}, {"print", {{' ', '~'}}},
            {"punct", {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}}},
            {"space", {{'\t', '\r'}, {' ', ' '}}}, {"upper", {{'A', 'Z'}}},
            {"word", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}, {'_', '_'}}},
            {"xdigit", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}}};
        auto it = g.find(name);
        if (it == g.end()) return false;
        r = it->second;
        return true;
    }
    static bool unicodeTable(const std::string& name, std::vector<std::pair<uint32_t, uint32_t>>& r) {
        r.clear();
        if (name == "Any") { r.push_back({0, 0x10FFFF}); return true; }
        for (uint32_t k = 0; k < ucd13::kNumCategories; k++)
            if (name == ucd13::kCategories[k].name) {
                for (uint32_t j = 0; j < ucd13::kCategories[k].n; j++) r.push_back({ucd13::kCategories[k].r[j].lo, ucd13::kCategories[k].r[j].hi});
                return true;
            }
        for (uint32_t k = 0; k < ucd13::kNumScripts; k++)
            if (name == ucd13::kScripts[k].name) {
                for (uint32_t j = 0; j < ucd13::kScripts[k].n; j++) r.push_back({ucd13::kScripts[k].r[j].lo, ucd13::kScripts[k].r[j].hi});
                return true;
            }
        return false;
    }

    // parseUnicodeClass: returns false when t[i..] is not \p / \P.
    bool parseUnicodeClass(const std::string& t, size_t& i, ClassItem& out) {
        if (!(flags & UnicodeGroups) || t.size() - i < 2 || t[i] != '\\' || (t[i + 1] != 'p' && t[i + 1] != 'P')) return false;
        bool neg = t[i + 1] == 'P';
        size_t j = i + 2;
        std::string name;
        size_t sz;
        const uint32_t c = decode_rune(t, j, &sz);
        if (c == 0xFFFD && sz == 1) throw SyntaxError();
        if (c != '{') {
            name = t.substr(j, sz);
            j += sz;
        } else {
            const size_t end = t.find('}', i);
            if (end == std::string::npos) { checkUTF8(t.substr(i)); throw SyntaxError(); }
            name = t.substr(i + 3, end - i - 3);
            checkUTF8(name);
            j = end + 1;
        }
        if (!name.empty() && name[0] == '^') { neg = !neg; name = name.substr(1); }
        if (!unicodeTable(name, out.base)) throw SyntaxError();
        out.fold = (flags & FoldCase) != 0;
        out.neg = neg;
        i = j;
        return true;
    }
    bool parsePerlClassEscape(const std::string& t, size_t& i, ClassItem& out) {
        if (!(flags & PerlX) || t.size() - i < 2 || t[i] != '\\') return false;
        const char c = t[i + 1];
        auto g = perlGroup(c);
        if (g.empty()) return false;
        out.base = g;
        out.fold = (flags & FoldCase) != 0;
        out.neg = c == 'D' || c == 'S' || c == 'W';
        i += 2;
        return true;
    }

    uint32_t parseClassChar(const std::string& t, size_t& i) {
        if (i >= t.size()) throw SyntaxError();   // missing closing ]
        if (t[i] == '\\') return parseEscape(t, i);
        return nextRune(t, i);
    }

    void parseClass(const std::string& t, size_t& i) {
        i++;   // [
        const int k = newRe(CharClass);
        if (i < t.size() && t[i] == '^') { at(k).negated = true; i++; }
        bool first = true;
        while (i >= t.size() || t[i] != ']' || first) {
            first = false;
            if (t.size() - std::min(t.size(), i) > 2 && t[i] == '[' && t[i + 1] == ':') {
                const size_t e = t.find(":]", i + 2);
                if (e != std::string::npos) {
                    std::string name = t.substr(i + 2, e - i - 2);
                    ClassItem it;
                    if (!name.empty() && name[0] == '^') { it.neg = true; name = name.substr(1); }
                    if (!posixGroup(name, it.base)) throw SyntaxError();
                    it.fold = (flags & FoldCase) != 0;
                    at(k).items.push_back(it);
                    i = e + 2;
                    continue;
                }
            }
            ClassItem it;
            if (parseUnicodeClass(t, i, it) || parsePerlClassEscape(t, i, it)) {
                at(k).items.push_back(it);
                continue;
            }
            const uint32_t lo = parseClassChar(t, i);
            uint32_t hi = lo;
            if (t.size() - std::min(t.size(), i) >= 2 && t[i] == '-' && t[i + 1] != ']') {
                i++;
                hi = parseClassChar(t, i);
                if (hi < lo) throw SyntaxError();
            }
            it.base = {{lo, hi}};
            it.fold = (flags & FoldCase) != 0;
            at(k).items.push_back(it);
        }
        i++;   // ]
        push(k);
    }

    // parsePerlFlags: t[i..] starts with "(?".
    void parsePerlFlags(const std::string& t, size_t& i) {
        if (t.size() - i > 4 && t[i + 2] == 'P' && t[i + 3] == '<') {
            const size_t end = t.find('>', i);
            if (end == std::string::npos) { checkUTF8(t.substr(i)); throw SyntaxError(); }
            const std::string name = t.substr(i + 4, end - i - 4);
            checkUTF8(name);
            if (name.empty()) throw SyntaxError();
            for (unsigned char ch : name) if (ch != '_' && !isalnum_(ch)) throw SyntaxError();
            numCap++;
            at(op(LeftParen)).cap = numCap;
            i = end + 1;
            return;
        }
        size_t j = i + 2;
        int fl = flags, sign = 1;
        bool sawFlag = false;
        while (j < t.size()) {
            const uint32_t c = nextRune(t, j);
            switch (c) {
                case 'i': fl |= FoldCase; sawFlag = true; break;
                case 'm': fl &= ~OneLine; sawFlag = true; break;
                case 's': fl |= DotNL; sawFlag = true; break;
                case 'U': fl |= NonGreedy; sawFlag = true; break;
                case '-':
                    if (sign < 0) throw SyntaxError();
                    sign = -1;
                    fl = ~fl;
                    sawFlag = false;
                    break;
                case ':':
                case ')':
                    if (sign < 0) {
                        if (!sawFlag) throw SyntaxError();
                        fl = ~fl;
                    }
                    if (c == ':') op(LeftParen);   // saves the flags in force before the group
                    flags = fl;
                    i = j;
                    return;
                default:
                    throw SyntaxError();
            }
        }
        throw SyntaxError();
    }

    int parse(const std::string& s) {
        whole = s;
        size_t i = 0;
        bool lastRepeat = false;
        while (i < s.size()) {
            bool repeatTok = false;
            const char c = s[i];
            if (c == '(') {
                if ((flags & PerlX) && s.size() - i >= 2 && s[i + 1] == '?') parsePerlFlags(s, i);
                else {
                    numCap++;
                    at(op(LeftParen)).cap = numCap;
                    i++;
                }
            } else if (c == '|') {
                parseVerticalBar();
                i++;
            } else if (c == ')') {
                parseRightParen();
                i++;
            } else if (c == '^') {
                op((flags & OneLine) ? BeginText : BeginLine);
                i++;
            } else if (c == '$') {
                op((flags & OneLine) ? EndText : EndLine);
                i++;
            } else if (c == '.') {
                op((flags & DotNL) ? AnyChar : AnyCharNotNL);
                i++;
            } else if (c == '[') {
                parseClass(s, i);
            } else if (c == '*' || c == '+' || c == '?') {
                i = repeat(c == '*' ? Star : c == '+' ? Plus : Quest, 0, 0, i + 1, lastRepeat, s);
                repeatTok = true;
            } else if (c == '{') {
                int mn = 0, mx = 0;
                size_t after;
                if (!parseRepeat(s, i, mn, mx, after)) {
                    literal('{');
                    i++;
                } else {
                    if (mn < 0 || mn > 1000 || mx > 1000 || (mx >= 0 && mn > mx)) throw SyntaxError();
                    i = repeat(Repeat, mn, mx, after, lastRepeat, s);
                    repeatTok = true;
                }
            } else if (c == '\\') {
                bool done = false;
                if ((flags & PerlX) && s.size() - i >= 2) {
                    switch (s[i + 1]) {
                        case 'A': op(BeginText); i += 2; done = true; break;
                        case 'b': op(WordBoundary); i += 2; done = true; break;
                        case 'B': op(NoWordBoundary); i += 2; done = true; break;
                        case 'C': throw SyntaxError();
                        case 'Q': {
                            const size_t e = s.find("\\E", i);
                            std::string lit = e == std::string::npos ? s.substr(i + 2) : s.substr(i + 2, e - i - 2);
                            i = e == std::string::npos ? s.size() : e + 2;
                            size_t j = 0;
                            while (j < lit.size()) literal(nextRune(lit, j));
                            done = true;
                            break;
                        }
                        case 'z': op(EndText); i += 2; done = true; break;
                    }
                }
                if (!done) {
                    ClassItem it;
                    if (parseUnicodeClass(s, i, it) || parsePerlClassEscape(s, i, it)) {
                        const int k = newRe(CharClass);
                        at(k).items.push_back(it);
                        push(k);
                    } else {
                        literal(parseEscape(s, i));
                    }
                }
            } else {
                literal(nextRune(s, i));
            }
            lastRepeat = repeatTok;
        }
        concat();
        if (swapVerticalBar()) stack.pop_back();
        alternate();
        if (stack.size() != 1) throw SyntaxError();   // missing closing )
        return stack[0];
    }
};

// ---- MatchString as position sets ------------------------------------------

class Matcher {
public:
    Matcher(const std::vector<Re>& pool, const std::string& text) : pool_(pool) {
        size_t i = 0;
        while (i < text.size()) {
            size_t w;
            runes_.push_back(decode_rune(text, i, &w));
            i += w;
        }
        n_ = runes_.size();
    }
    using Set = std::vector<char>;   // positions 0..n (rune boundaries)

    bool any(int root) {
        Set all(n_ + 1, 1);
        Set e = eval(root, all);
        for (char c : e) if (c) return true;
        return false;
    }

private:
    const std::vector<Re>& pool_;
    std::vector<uint32_t> runes_;
    size_t n_ = 0;

    static bool isWord(int64_t r) {
        return r >= 0 && (('0' <= r && r <= '9') || ('a' <= r && r <= 'z') || ('A' <= r && r <= 'Z') || r == '_');
    }
    // EmptyOpContext(r1, r2) at position p
    bool assertion(int op, size_t p) const {
        const int64_t r1 = p == 0 ? -1 : (int64_t)runes_[p - 1];
        const int64_t r2 = p == n_ ? -1 : (int64_t)runes_[p];
        switch (op) {
            case BeginText: return r1 < 0;
            case EndText: return r2 < 0;
            case BeginLine: return r1 < 0 || r1 == '\n';
            case EndLine: return r2 < 0 || r2 == '\n';
            case WordBoundary: return isWord(r1) != isWord(r2);
            case NoWordBoundary: return isWord(r1) == isWord(r2);
        }
        return false;
    }
    bool char_ok(const Re& re, uint32_t c) const {
        switch (re.op) {
            case AnyChar: return true;
            case AnyCharNotNL: return c != '\n';
            case Literal:
                if (!(re.flags & FoldCase)) return c == re.rune;
                return scf(c) == scf(re.rune);
            case CharClass: {
                bool in = false;
                for (auto& it : re.items) if (item_has(it, c)) { in = true; break; }
                return in != re.negated;
            }
        }
        return false;
    }
    static bool empty(const Set& s) {
        for (char c : s) if (c) return false;
        return true;
    }
    static void unite(Set& a, const Set& b) {
        for (size_t k = 0; k < a.size(); k++) a[k] |= b[k];
    }
    Set closure(int sub, Set reach) {   // zero or more sub's from reach
        Set frontier = reach;
        while (!empty(frontier)) {
            Set nx = eval(sub, frontier), fresh(n_ + 1, 0);
            for (size_t k = 0; k <= n_; k++) if (nx[k] && !reach[k]) { fresh[k] = 1; reach[k] = 1; }
            frontier = fresh;
        }
        return reach;
    }
    Set eval(int k, const Set& from) {
        const Re& re = pool_[k];
        Set out(n_ + 1, 0);
        switch (re.op) {
            case NoMatch: return out;
            case EmptyMatch: return from;
            case Literal: case CharClass: case AnyChar: case AnyCharNotNL:
                for (size_t p = 0; p < n_; p++) if (from[p] && char_ok(re, runes_[p])) out[p + 1] = 1;
                return out;
            case BeginLine: case EndLine: case BeginText: case EndText: case WordBoundary: case NoWordBoundary:
                for (size_t p = 0; p <= n_; p++) if (from[p] && assertion(re.op, p)) out[p] = 1;
                return out;
            case Capture: return eval(re.sub[0], from);
            case Concat: {
                Set cur = from;
                for (int s : re.sub) cur = eval(s, cur);
                return cur;
            }
            case Alternate:
                for (int s : re.sub) unite(out, eval(s, from));
                return out;
            case Star: return closure(re.sub[0], from);
            case Plus: return closure(re.sub[0], eval(re.sub[0], from));
            case Quest: out = from; unite(out, eval(re.sub[0], from)); return out;
            case Repeat: {
                Set cur = from;
                for (int r = 0; r < re.min; r++) cur = eval(re.sub[0], cur);
                if (re.max < 0) return closure(re.sub[0], cur);
                out = cur;
                for (int r = re.min; r < re.max && !empty(cur); r++) {
                    cur = eval(re.sub[0], cur);
                    unite(out, cur);
                }
                return out;
            }
        }
        return out;
    }
};

// regexp.Compile: false on a syntax error.
inline bool compile(const std::string& expr, std::vector<Re>* pool, int* root) {
    GoParser p;
    try {
        *root = p.parse(expr);
    } catch (const SyntaxError&) {
        return false;
    }
    *pool = std::move(p.pool);
    return true;
}

inline bool match_string(const std::vector<Re>& pool, int root, const std::string& text) {
    return Matcher(pool, text).any(root);
}

}  // namespace orare
