"""Regenerate tests/golden/plan_apply.json from the oracle (self-derived golden
vectors for the plan applier fit check; inputs are regenerated from seeds).

Not reference outputs (Go cannot run here): they freeze the
oracle's per-node evaluateNodePlan outcomes so the HIP planner is checked
against committed data and any change of the oracle shows up as a diff. The
oracle itself is pinned by plan_apply_test.go / funcs_test.go KATs.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nomad_amd.synth_plan import random_case, system_plan  # noqa: E402
from oracle import plan_apply as O  # noqa: E402

RANDOM_SEEDS = list(range(40))
SYSTEM = dict(n=3000, seed=17)


def outcomes(nodes, allocs, plan):
    ids, fits, why = O.evaluate_plan_placements(O.Snapshot(nodes, allocs), plan)
    return [[i, f, w] for i, f, w in zip(ids, fits, why)]


def main():
    out = {"random_case": {str(s): outcomes(*random_case(s)) for s in RANDOM_SEEDS},
           "system_plan": dict(SYSTEM, outcomes=outcomes(*system_plan(SYSTEM["n"], SYSTEM["seed"])))}
    path = os.path.join(ROOT, "tests", "golden", "plan_apply.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
