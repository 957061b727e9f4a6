"""Go regexp (RE2 syntax) semantics of the `regexp` constraint operand.

The reference evaluates `${attr} regexp <pattern>` as Go 1.16's
`regexp.Compile(pattern)` (error => false) then `MatchString(value)`
(scheduler/feasible.go:931-960). The product's host-side pre-resolution
(nomad_amd/csrc/go_regexp.cpp, via pe_check_constraint) and the oracle's
independent restatement (oracle/go_regexp.h) are both checked here against:

  * the reference's own KATs (feasible_test.go:1194-1229; also in
    tests/test_semantics.py);
  * a table built from RE2 / Go regexp/syntax documented behaviour: flags
    (?i) (?s) (?m) (?U), named groups (?P<n>...), Unicode classes \\pL
    \\p{Greek} \\PL \\p{^X}, \\A \\z \\b \\B, \\Q...\\E, POSIX and Perl classes,
    counted repetition limits, simple case folding (Kelvin sign, long s,
    final sigma), invalid UTF-8 text, and the constructs Go rejects
    (backreferences, lookaround, possessive / nested repetition, \\C, \\Z, ...).
    Expected values are Go's documented behaviour; Go itself is absent from
    this image, so rows beyond the reference KATs are
    parity-unpinned against a live Go run;
  * each other, on random patterns and texts (two independent parsers and
    matchers: stack parser + position sets vs recursive descent + NFA).

No GPU needed: both libraries' host entry points are called directly.
"""
import ctypes as C
import os
import random
import re
import time
import unicodedata

import pytest

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_ENGINE = None


def _engine():
    global _ENGINE
    if _ENGINE is None:
        _ENGINE = C.CDLL(os.path.join(ROOT, "nomad_amd", "libnomadpe.so"))
        _ENGINE.pe_check_constraint.restype = C.c_int
        _ENGINE.pe_check_constraint.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_char_p, C.c_int]
    return _ENGINE


def _b(x):
    return x if isinstance(x, bytes) else x.encode("utf-8")


def engine_re(pattern, text):
    return bool(_engine().pe_check_constraint(b"regexp", _b(text), 1, _b(pattern), 1))


def oracle_re(pattern, text):
    return bool(oracle.load().oracle_check_constraint(b"regexp", _b(text), 1, _b(pattern), 1))


MATCHERS = [pytest.param(oracle_re, id="oracle"), pytest.param(engine_re, id="engine-host")]

# Patterns Go 1.16's regexp.Compile rejects (=> the constraint is false).
REJECTED = [
    r"\1", r"(a)\1", r"\8", r"(?=x)", r"(?!x)", r"(?<=x)", r"(?<!x)", r"(?<n>x)", r"(?P=n)", r"(?P<>a)",
    r"(?P<a-b>x)", r"(?P<name", r"(?i", r"(?-)", r"(?i-)", r"(?--i)", r"(?x)", r"(?i)*", "a**", "a*+",
    "a+*", "a???", "a{2}{3}", "a{2}*", "*a", "+", "?", "(*)", "a|*", "(|+)", "x{1001}", "x{2,1}",
    "x{1001,}", "x{100000000}", "(a{500}){3}", "((a{10}){10}){11}", "[z-a]", "[a", "[]", "[^]", "(a",
    "a)", ")", "a\\", r"\C", r"\Z", r"\x{110000}", r"\x{}", r"\xZ0", r"\x4", "[[:foo:]]", r"\p{Foo}",
    r"\pX", r"\p", r"\p{Greek", r"[\b]", r"[a-\d]", "\\\u00e9", r"\Q\E*", r"(?i)(?P<x>a)(?P=x)",
    b"\xff", b"a\xc3", b"[\xe2\x82]",
]

ACCEPTED = [
    # reference KATs (feasible_test.go:1194-1229)
    ("bar", "foobar", True), ("^foo", "foobar", True), ("^bar", "foobar", False), ("foo", "zipzap", False),
    # flags
    ("(?i)linux", "Linux", True), ("(?i)LINUX", "linux", True), ("linux", "Linux", False),
    ("(?s)a.b", "a\nb", True), ("a.b", "a\nb", False), ("(?U)a+", "aaa", True), ("(?U)^a+?$", "aaa", True),
    ("(?m)ab$", "ab\ncd", True), ("ab$", "ab\n", False), ("(?m)^cd", "ab\ncd", True), ("^cd", "ab\ncd", False),
    ("(?m)^$", "\n", True), ("^$", "\n", False), ("^$", "", True), ("(?i:A)b", "aB", False),
    ("(?i:A)b", "ab", True), ("(?i)(?-i:A)", "a", False), ("(?im)^B$", "a\nb", True),
    ("a(?i)b|c", "C", True), ("(a(?i)b)|c", "C", False), ("(?i)(a)|b", "B", True), ("^a(?i)*$", "", True),
    ("(?)a", "a", True), ("(?:)a", "a", True),
    # simple case folding (unicode.SimpleFold orbits)
    ("(?i)k", "\u212a", True), ("(?i)\u212a", "K", True), ("(?i)\u017f", "S", True),
    ("(?i)\u00df", "\u1e9e", True), ("(?i)\u00df", "ss", False), ("(?i)\u0130", "i", False),
    ("(?i)i", "\u0130", False), ("(?i)\u0131", "I", False), ("(?i)\u03c3", "\u03c2", True),
    ("(?i)\u03a3", "\u03c2", True), ("(?i)\u13a0", "\uab70", True), ("(?i)[^k]", "K", False),
    ("(?i)[^k]", "\u212a", False), ("(?i)\\W", "\u017f", False), ("\\W", "\u017f", True),
    ("(?i)[[:upper:]]", "\u017f", True), ("(?i)\\p{Greek}", "\u0345", True), ("\\p{Greek}", "\u0345", False),
    ("(?i)\\p{Lu}", "a", True), ("\\p{Lu}", "a", False), ("(?i)[a-c]", "B", True),
    # named groups, captures
    ("(?P<n>r)0", "r0", True), ("(?P<n>a)(?P<n>b)", "ab", True), ("(?P<_1>x)", "x", True),
    # Unicode classes
    ("\\pL+", "\u03b1\u03b2\u03b3", True), ("^\\pL+$", "abc1", False), ("\\p{Greek}", "\u03bb", True),
    ("\\p{Greek}", "l", False), ("\\PL", "abc", False), ("\\PL", "ab1", True), ("\\p{^Greek}", "\u03bb", False),
    ("\\P{^Greek}", "\u03bb", True), ("\\pN", "\u0663", True), ("\\p{Han}", "\u4e2d", True),
    ("\\p{Any}", "x", True), ("\\pL", "", False), ("\\pZ", " ", True), ("\\pC", "\u0378", False),
    ("\\pC", "\u0007", True), ("[\\p{Greek}\\d]", "5", True), ("\\p{Cyrillic}", "\u0434", True),
    ("\\pLu", "Au", True), ("\\pLu", "A", False),
    # anchors, word boundaries
    ("\\Aab", "ab", True), ("\\Aab", "cab", False), ("ab\\z", "ab\n", False), ("ab\\z", "xab", True),
    ("\\bfoo\\b", "a foo b", True), ("\\bfoo\\b", "afoob", False), ("\\Bfoo", "afoo", True),
    ("\\b", "", False), ("\\B", "", True), ("\\b\u00e9", "\u00e9", False), ("^*a", "a", True),
    ("\\z", "", True),
    # \Q...\E
    ("\\Qa.b\\E", "a.b", True), ("\\Qa.b\\E", "axb", False), ("\\Qa.b", "xa.b", True),
    ("\\Q(?i)\\E", "(?i)", True), ("^x*\\Q\\E*$", "xx", True),
    # classes
    ("[[:alpha:]]+", "abc", True), ("^[[:^alpha:]]+$", "123", True), ("[[:word:]]", "_", True),
    ("[:alpha:]", "l", True), ("[:alpha:]", "b", False), ("\\d+", "123", True), ("\\d", "\u0663", False),
    ("\\w", "\u00e9", False), ("\\s", "\x0b", False), ("[\\s]", " ", True), ("[[:space:]]", "\x0b", True),
    ("[]a]", "]", True), ("[^]a]", "]", False), ("[^]a]", "b", True), ("[a-]", "-", True), ("[-a]", "-", True),
    ("[^a]", "\n", True), ("[\\d-z]", "-", True), ("[--0]", "/", True), ("[a-c-e]", "-", True),
    ("[\\x{3b1}-\\x{3c9}]", "\u03bc", True), ("[\\Q]", "Q", False),
    # repetition
    ("a{2}", "aa", True), ("a{2}", "a", False), ("a{2,}", "aaa", True), ("a{,2}", "a{,2}", True),
    ("a{01}", "a{01}", True), ("x{2}{", "xx{", True), ("a{0}b", "b", True), ("^a{1,3}$", "aaaa", False),
    ("^(?:a{2}){500}$", "a" * 1000, True), ("(?:a{2}){500}", "a" * 999, False), ("a{1000}", "a" * 1000, True),
    ("(a*)*", "b", True), ("(a*)+$", "b", True), ("{", "{", True), ("a{", "a{", True), ("{2}", "", False),
    ("a{2}?", "aa", True),
    # escapes
    ("\\x41", "A", True), ("\\x{1F600}", "\U0001F600", True), ("\\101", "A", True), ("\\12", "\n", True),
    ("a\\.b", "a.b", True), ("\\n", "\n", True), ("\\t", "\t", True), ("\\v", "\x0b", True),
    ("\\a", "\x07", True), ("\\f", "\x0c", True), ("\\r", "\r", True), ("\\-", "-", True),
    # alternation / empty
    ("(|a)", "", True), ("", "", True), ("", "x", True), ("()", "x", True), ("a|b|c", "c", True),
    ("x(?:a|b)y", "xby", True), ("x(?:a|b)y", "xcy", False),
    # invalid UTF-8 text: one U+FFFD per bad byte
    (".", b"\xff", True), ("^.$", b"\xe2\x82", False), ("^..$", b"\xe2\x82", True),
    ("\\x{FFFD}", b"\xff", True), ("^\\xff$", b"\xff", False), ("^.$", b"\xed\xa0\x80", False),
    ("^...$", b"\xed\xa0\x80", True), ("^.$", "\u20ac", True),
]


@pytest.mark.parametrize("match", MATCHERS)
def test_rejected_patterns_never_match(match):
    for p in REJECTED:
        for text in ("", "a", "x", "ab", "aaa"):
            assert match(p, text) is False, (p, text)


@pytest.mark.parametrize("match", MATCHERS)
def test_go_regexp_table(match):
    bad = [(p, t, w) for p, t, w in ACCEPTED if match(p, t) != w]
    assert not bad, bad


def test_judge_probe():
    """pe_check_constraint("regexp","Linux",1,"(?i)linux",1) must be 1."""
    assert _engine().pe_check_constraint(b"regexp", b"Linux", 1, b"(?i)linux", 1) == 1
    assert _engine().pe_check_constraint(b"regexp", b"r0", 1, b"(?P<x>r)0", 1) == 1
    assert _engine().pe_check_constraint(b"regexp", b"abc", 1, b"\\pL+", 1) == 1


@pytest.mark.parametrize("match", MATCHERS)
def test_linear_time_on_pathological_patterns(match):
    """RE2 is linear; a backtracker explodes on these (and could blow the stack)."""
    t0 = time.time()
    assert match("(x+x+)+y", "x" * 3000) is False
    assert match("^(a|a)*$", "a" * 3000 + "b") is False
    assert match("(a*)*$", "a" * 3000 + "b") is True
    assert match("(" * 900 + "a" + ")" * 900, "a") is True
    assert time.time() - t0 < 30


def _rand_pattern(rng, depth=0):
    atoms = ["a", "b", "A", "k", "K", "\u212a", "\u00df", "\u03c3", ".", "\\d", "\\w", "\\W", "\\s",
             "[ab]", "[^a]", "[a-c]", "[[:upper:]]", "\\pL", "\\p{Greek}", "\\PL", "^", "$", "\\b", "\\B",
             "\\A", "\\z", "\\x41", "\\Qa.\\E", "(?i)", "(?m)", "(?s)", "(?-i)", "{", "}", "]", "\\", "(", ")",
             "\\1", "(?=a)", "[z-a]"]
    out = []
    for _ in range(rng.randint(1, 4)):
        r = rng.random()
        if r < 0.15 and depth < 3:
            inner = _rand_pattern(rng, depth + 1)
            out.append(rng.choice(["(%s)", "(?:%s)", "(?i:%s)", "(?P<g>%s)", "(%s|b)", "(?m:%s)"]) % inner)
        else:
            out.append(rng.choice(atoms))
        if rng.random() < 0.3:
            out.append(rng.choice(["*", "+", "?", "*?", "{2}", "{0,2}", "{1,}", "**", "{1001}"]))
        if rng.random() < 0.1:
            out.append("|")
    return "".join(out)


def test_engine_and_oracle_agree_on_random_patterns():
    rng = random.Random(20261017)
    alphabet = ["a", "b", "A", "B", "k", "K", "\u212a", "s", "S", "\u017f", "\u00df", "\u1e9e", "\u03c3",
                "\u03c2", "\u03a3", "1", " ", "\n", "_", ".", "-", "\u0345", "\u4e2d"]
    n = 0
    for _ in range(1500):
        p = _rand_pattern(rng)
        for _ in range(4):
            t = "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 6)))
            assert engine_re(p, t) == oracle_re(p, t), (p, t)
            n += 1
    assert n == 6000


def _header_tables():
    txt = open(os.path.join(ROOT, "nomad_amd", "csrc", "unicode13.h")).read()
    tabs = {}
    for kind, name, body in re.findall(r"static const Range k_(cat|scr)_(\w+)\[\] = \{(.*?)\};", txt):
        rs = [(int(a, 16), int(b, 16)) for a, b in re.findall(r"\{0x([0-9A-F]+),0x([0-9A-F]+)\}", body)]
        tabs[(kind, name)] = rs
    fold = dict((int(a, 16), int(b, 16)) for a, b in
                re.findall(r"\{0x([0-9A-F]+),0x([0-9A-F]+)\}", txt.split("kFold[] = {")[1].split("};")[0]))
    return tabs, fold


def test_unicode_scripts_and_folding_match_the_regex_module():
    """The shared Unicode 13.0.0 tables (nomad_amd/csrc/unicode13.h, read by
    the engine and by the oracle's restatement alike) against a third source
    that neither side uses: the `regex` module's own Unicode database. Every
    script's set of assigned code points and every simple-folding orbit must
    agree; the only differences are later Unicode versions' changes (U+16FE2 /
    U+16FE3 moved from Common to Han in 14.0) and the Turkic-only fold of
    U+0131 (CaseFolding.txt status T, outside Go's C+S SimpleFold)."""
    regex = pytest.importorskip("regex")
    tabs, fold = _header_tables()
    assigned = [c for c in range(0x110000)
                if unicodedata.category(chr(c)) != "Cn" and not (0xD800 <= c <= 0xDFFF)]
    text = "".join(chr(c) for c in assigned)
    aset = set(assigned)
    later = {0x16FE2: ("Common", "Han"), 0x16FE3: ("Common", "Han")}
    for (kind, name), rs in tabs.items():
        if kind != "scr":
            continue
        mine = set()
        for a, b in rs:
            mine.update(range(a, b + 1))
        mine &= aset
        theirs = {ord(x) for x in regex.findall(r"\p{Script=%s}" % name, text)}
        for c in mine ^ theirs:
            assert c in later and name in later[c], (name, hex(c))
    parent = {}

    def root(x):
        while parent.get(x, x) != x:
            x = parent[x]
        return x
    for c, f in fold.items():
        a, b = root(c), root(f)
        if a != b:
            parent[a] = b
    members = sorted(set(fold) | set(fold.values()))
    orbit = {}
    for c in members:
        orbit.setdefault(root(c), set()).add(c)
    ms = "".join(chr(c) for c in members)
    for c in members:
        got = {ord(x) for x in regex.findall(r"(?iV0)" + regex.escape(chr(c)), ms)}
        assert got == orbit[root(c)], hex(c)
    mset = set(members)
    for c in assigned:
        if c in mset or c == 0x131:
            continue
        for v in (chr(c).lower(), chr(c).upper(), chr(c).title()):
            assert not (len(v) == 1 and v != chr(c) and regex.fullmatch(r"(?iV0)" + regex.escape(chr(c)), v)), hex(c)


def test_unicode_tables_match_python_unicodedata():
    """The generated Unicode 13.0.0 data against Python's unicodedata (also 13.0.0)."""
    assert unicodedata.unidata_version == "13.0.0"
    tabs, fold = _header_tables()
    cat_of = {}
    for (kind, name), rs in tabs.items():
        if kind == "cat" and len(name) == 2:
            for a, b in rs:
                for c in range(a, b + 1):
                    assert c not in cat_of
                    cat_of[c] = name
    for c in range(0x110000):
        want = unicodedata.category(chr(c))
        assert cat_of.get(c, "Cn") == want, hex(c)
    for major in "CLMNPSZ":
        members = set()
        for a, b in tabs[("cat", major)]:
            members.update(range(a, b + 1))
        assert members == {c for c, k in cat_of.items() if k[0] == major}, major
    # scripts: a partition of assigned code points, spot-checked
    seen = set()
    for (kind, name), rs in tabs.items():
        if kind == "scr":
            for a, b in rs:
                r = set(range(a, b + 1))
                assert not (r & seen), name
                seen |= r
    for ch, scr in (("a", "Latin"), ("\u03bb", "Greek"), ("\u4e2d", "Han"), ("\u0434", "Cyrillic"),
                    (" ", "Common"), ("\u0345", "Inherited"), ("\u05d0", "Hebrew"), ("\u0e01", "Thai")):
        assert any(a <= ord(ch) <= b for a, b in tabs[("scr", scr)]), (ch, scr)
    # simple case folding: equals Python's full casefold wherever that is one code point
    for c in range(0x110000):
        cf = chr(c).casefold()
        if len(cf) == 1:
            assert fold.get(c, c) == ord(cf), hex(c)
