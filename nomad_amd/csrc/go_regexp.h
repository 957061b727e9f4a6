// Go regexp semantics for the `regexp` constraint operand (product code, host side).
//
// The reference evaluates `regexp` constraints with Go's standard library:
// `regexp.Compile(rVal)` then `re.MatchString(lVal)`, a compile error meaning
// "no match" (scheduler/feasible.go:931-960; the device-attribute form at
// feasible.go:1334-1447 goes through the same call). Go's package is RE2
// syntax with the syntax.Perl flags (ClassNL | OneLine | PerlX |
// UnicodeGroups) as of Go 1.16.7 (.circleci/config.yml:527): Unicode 13.0.0
// classes, simple case folding, no backreferences or lookaround.
//
// compile() accepts exactly the patterns Go 1.16's regexp/syntax parser
// accepts (see go_regexp.cpp for the rules: flag groups, named captures,
// repeat sizes incl. repeatIsValid, class syntax, escapes, UTF-8 checks) and
// builds a Thompson NFA over Unicode code points. match() is Go's
// MatchString: does some substring of the UTF-8 text, split at the same rune
// boundaries Go's decoder uses (invalid bytes are U+FFFD of width 1), match
// the pattern. It simulates the NFA over rune positions (Pike-style state
// sets), so time is linear in |text| x |program| and no pattern can recurse
// on the host stack.
#pragma once
#include <cstdint>
#include <memory>
#include <string>

namespace pe {
namespace gore {

struct Prog;

enum CompileStatus {
    kOk = 0,
    kSyntaxError = 1,   // Go's regexp.Compile returns an error
    kTooLarge = 2,      // accepted by Go, but the expanded program exceeds kMaxInst
};

constexpr uint32_t kMaxInst = 1u << 23;

// regexp.Compile(expr): null unless *status == kOk.
std::shared_ptr<const Prog> compile(const std::string& expr, int* status);

// (*Regexp).MatchString(text)
bool match(const Prog& prog, const std::string& text);

// Convenience: compile + match, false on any compile failure.
bool match_string(const std::string& expr, const std::string& text);

}  // namespace gore
}  // namespace pe
