"""Regenerate tests/golden/*.json from the oracle (self-derived golden vectors).

These fixtures are NOT reference outputs (the Go reference cannot be built
here); they freeze the oracle's results on seeded inputs so the
engine is checked against committed data on the GPU box and any change of the
oracle itself shows up as a diff. Inputs are regenerated from the seeds.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nomad_amd import synth  # noqa: E402
from oracle.oracle import OracleGenericStack, OracleSystemStack  # noqa: E402

CASES = {
    "c1_mock_count10": dict(gen="c1", n=100, seed=42, perm_seed=1, count=10),
    "c2_binpack_2k": dict(gen="c2", n=2000, seed=42, perm_seed=5, count=400),
    "c3_spread_affinity_1k": dict(gen="c3", n=1000, seed=7, perm_seed=3, count=150),
    "c5_devices_preempt_600": dict(gen="c5", n=600, seed=4, perm_seed=9, count=200, busy=0.9, preempt=True),
}


def build(case):
    if case["gen"] == "c1":
        nodes, allocs = synth.cluster_c1(case["n"], seed=case["seed"])
        job = synth.mock_job(count=case["count"])
    elif case["gen"] == "c2":
        nodes, allocs = synth.cluster_c2(case["n"], seed=case["seed"])
        job = synth.job_c2(case["count"])
    elif case["gen"] == "c5":
        nodes, allocs = synth.cluster_c5(case["n"], seed=case["seed"], busy=case["busy"])
        job = synth.job_c5(case["count"])
    else:
        nodes, allocs = synth.cluster_c3(case["n"], seed=case["seed"])
        job = synth.job_c3(case["count"])
    perm = synth.shuffle(len(nodes), case["perm_seed"])
    return nodes, allocs, job, perm


def config(case):
    from nomad_amd.structs import SchedulerConfig
    return SchedulerConfig(preempt_service=bool(case.get("preempt")))


def run(name, case):
    nodes, allocs, job, perm = build(case)
    st = OracleGenericStack(config=config(case))
    st.SetState(nodes, allocs)
    st.SetJob(job)
    limit = st.SetNodes(list(perm))
    res = st.Place(0, case["count"])
    return {"case": case, "limit": limit,
            "placements": [{"node_id": r.node.id if r.node else None, "row": r.row,
                            "final_score": r.final_score.hex(), "scores": [s.hex() for s in r.scores],
                            "evaluated": r.nodes_evaluated, "filtered": r.nodes_filtered,
                            "exhausted": r.nodes_exhausted, "offset": r.new_offset,
                            "preempted": sorted(r.preempted), "device_offers": r.device_offers} for r in res]}


if __name__ == "__main__":
    out = os.path.join(ROOT, "tests", "golden")
    for name, case in CASES.items():
        with open(os.path.join(out, name + ".json"), "w") as f:
            json.dump(run(name, case), f, indent=0)
        print("wrote", name)
