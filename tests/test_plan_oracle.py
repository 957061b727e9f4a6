"""The C++ plan-applier restatement (oracle/plan_oracle.cpp: evaluateNodePlan /
AllocsFit / NetworkIndex / DeviceAccounter over pe_planner_*'s POD inputs,
nomad/plan_apply.go:611-674, nomad/structs/funcs.go:148-211) against the
Python restatement the reference's own tests pin (tests/test_plan_apply.py):
the reference KATs, the committed golden outcomes, 120 random edge-heavy
cases, big-key nodes and a commit chain. CPU only: it is bench.py's
plan_apply cpu_baseline."""
import random

import pytest

from nomad_amd.plan import Plan, PlanAlloc, assemble_result
from nomad_amd.synth_plan import random_case, system_plan
from oracle import plan_apply as O
from oracle.oracle import OraclePlanner
from tests.test_plan_apply import KATS, _codes_to_pairs, _golden


@pytest.mark.parametrize("kat", KATS, ids=lambda f: f.__name__)
def test_cpp_oracle_reference_kats(kat):
    nodes, allocs, plan, expect = kat()
    pl = OraclePlanner()
    pl.set_state(nodes, allocs)
    for nid, (fit, why) in expect.items():
        assert pl.evaluate_node_plan(plan, nid) == (fit, why), nid
    snap = O.Snapshot(nodes, allocs)
    assert pl.evaluate_plan_placements(plan) == \
        assemble_result(plan, *O.evaluate_plan_placements(snap, plan), snap.alloc_by_id)


def test_cpp_oracle_random_and_big_keys():
    seen = set()
    for seed, kw in [(s, {}) for s in range(120)] + [(s, dict(n_nodes=16, max_allocs=6, big_keys=True))
                                                      for s in range(200, 220)]:
        nodes, allocs, plan = random_case(seed, **kw)
        pl = OraclePlanner()
        pl.set_state(nodes, allocs)
        ep = pl.encode(plan)
        got = _codes_to_pairs(pl.evaluate(ep))
        ids, fits, why = O.evaluate_plan_placements(O.Snapshot(nodes, allocs), plan)
        assert ids == ep.node_ids and got == list(zip(fits, why)), seed
        seen |= {w for _, w in got}
    assert {"", "node does not exist", "node is not ready for placements", "node is not eligible", "cores", "cpu",
            "memory", "disk", "reserved port collision", "device oversubscribed"} <= seen, seen


def test_cpp_oracle_golden():
    g = _golden()
    pl = OraclePlanner()
    for seed, want in g["random_case"].items():
        nodes, allocs, plan = random_case(int(seed))
        pl.set_state(nodes, allocs)
        ep = pl.encode(plan)
        assert [[nid, f, w] for nid, (f, w) in zip(ep.node_ids, _codes_to_pairs(pl.evaluate(ep)))] == want, seed
    sp = g["system_plan"]
    nodes, allocs, plan = system_plan(sp["n"], sp["seed"])
    pl.set_state(nodes, allocs)
    ep = pl.encode(plan)
    assert [[nid, f, w] for nid, (f, w) in zip(ep.node_ids, _codes_to_pairs(pl.evaluate(ep)))] == sp["outcomes"]


def test_cpp_oracle_commit_chain():
    rng = random.Random(7)
    nodes, allocs, plan = random_case(1000, n_nodes=32)
    pl = OraclePlanner()
    pl.set_state(nodes, allocs)
    snap = O.Snapshot(nodes, allocs)
    for step in range(6):
        res = pl.evaluate_plan_placements(plan)
        ref = assemble_result(plan, *O.evaluate_plan_placements(snap, plan), snap.alloc_by_id)
        assert res == ref, step
        pl.apply(plan, res)
        snap.apply(plan, ref)
        live = list(snap.by_id.values())
        plan = Plan()
        for n in rng.sample(nodes, 20):
            mine = [a for a in live if a.node_id == n.id]
            placed = [PlanAlloc(id="s%d-%s" % (step, n.id), node_id=n.id, cpu_shares=rng.choice([500, 1500]),
                                memory_mb=256, disk_mb=150)]
            if mine and rng.random() < 0.4:
                plan.node_update[n.id] = [rng.choice(mine)]
            plan.node_allocation[n.id] = placed
