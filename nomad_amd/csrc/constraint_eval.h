// Host-side constraint semantics for pre-resolution (product code).
//
// The engine evaluates constraints once per distinct (class | value) on the
// host and ships the verdicts to HBM as class / value tables. This header
// implements the operand semantics of scheduler/feasible.go:785-1024
// (checkConstraint and friends), go-version constraint matching
// (github.com/hashicorp/go-version @ 2046c9d0f0b0, go.mod:75) and the semver
// operand (helper/constraints/semver/constraints.go). Version strings are
// parsed by a hand-written scanner equivalent to go-version's
// VersionRegexpRaw / SemverRegexpRaw.
#pragma once
#include <cstdint>
#include <string>
#include <vector>
#include <unordered_map>
#include <memory>

#include "go_regexp.h"

namespace pe {

// A resolved constraint target: Go's (interface{}, found). `nil` only for an
// unknown ${...} interpolation; a missing attribute is ("", false).
struct Target {
    bool nil = true;
    bool found = false;
    std::string value;
};

struct SemVer {
    std::vector<int64_t> seg;   // padded to >= 3
    int specified = 0;
    std::string pre, meta;
};

// go-version NewVersion (semver=false) / NewSemver (semver=true)
bool parse_version(const std::string& s, bool semver, SemVer* out);
int compare_versions(const SemVer& a, const SemVer& b);

struct VersionConstraint {
    int op;        // 0 = 1 != 2 > 3 < 4 >= 5 <= 6 ~>
    SemVer v;
};
bool parse_version_constraints(const std::string& s, bool semver, std::vector<VersionConstraint>* out);
bool check_version_constraints(const std::vector<VersionConstraint>& cs, const SemVer& v, bool semver);

// Typed device attribute (plugins/shared/structs/attribute.go:85-101).
struct DevAttr {
    enum Kind : uint8_t { kNone, kInt, kFloat, kString, kBool } kind = kNone;
    int64_t i = 0;
    double f = 0;
    bool b = false;
    std::string s;
    std::string unit;
};
// psstructs.ParseAttribute (attribute.go:55-103)
DevAttr parse_dev_attr(const std::string& in);
// Attribute.Compare (attribute.go:322-385); *ok = comparable
int compare_dev_attr(const DevAttr& a, const DevAttr& b, bool* ok);

class ConstraintEvaluator {
public:
    // checkConstraint (feasible.go:785-820)
    bool check(const std::string& op, const Target& l, const Target& r);
    // checkAttributeConstraint (feasible.go:1334-1447), also checkAttributeAffinity
    bool check_attr(const std::string& op, const DevAttr& l, bool lf, const DevAttr& r, bool rf);

private:
    bool version_match(bool semver, const Target& l, const Target& r);
    bool regexp_match(const Target& l, const Target& r);
    std::unordered_map<std::string, std::shared_ptr<std::vector<VersionConstraint>>> ver_cache_[2];
    // regexp.Compile results per pattern (ctx.RegexpCache(), feasible.go:945-957);
    // null = the pattern does not compile (Go returns false for it)
    std::unordered_map<std::string, std::shared_ptr<const gore::Prog>> re_cache_;
};

bool target_escapes(const std::string& t);   // node_class.go:120-132

}  // namespace pe
