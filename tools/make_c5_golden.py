"""tests/golden/c5_bench_shape.json.gz: the oracle's 1000 placements of
bench.py's C5 workload (section_c5: cluster_c5(50000, seed=5, busy=0.99),
job_c5(1000), shuffle(.., 77), service preemption on).

Self-derived from the oracle (the Go reference cannot run here, SURVEY.md
§8c), like tools/make_golden.py: the oracle takes ~10 minutes on one core for
this evaluation (628 Selects with Preempt over 50k nodes), too long for a GPU
test, so the GPU test compares the engine with this frozen oracle output and
tests/test_golden.py re-derives its first placements on the CPU to catch drift.
The loop is the caller's itself (Select, Preempt retry on nil, commit with
the preempted set); the plain nil before each retry is kept too, so the
fixture answers both engine protocols, the served records included.
"""
import gzip
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nomad_amd import synth  # noqa: E402
from nomad_amd.structs import SchedulerConfig  # noqa: E402
from oracle.oracle import OracleGenericStack  # noqa: E402

CASE = dict(n=50000, seed=5, busy=0.99, perm_seed=77, count=1000)
OUT = os.path.join(ROOT, "tests", "golden", "c5_bench_shape.json.gz")


def build(case=CASE):
    nodes, allocs = synth.cluster_c5(case["n"], seed=case["seed"], busy=case["busy"])
    job = synth.job_c5(case["count"])
    perm = synth.shuffle(len(nodes), case["perm_seed"])
    return nodes, allocs, job, perm, SchedulerConfig(preempt_service=True)


def record(r):
    return {"row": r.row, "final_score": r.final_score.hex(), "scores": [s.hex() for s in r.scores],
            "evaluated": r.nodes_evaluated, "filtered": r.nodes_filtered, "exhausted": r.nodes_exhausted,
            "offset": r.new_offset, "preempted": list(r.preempted), "device_offers": list(r.device_offers)}


def main():
    nodes, allocs, job, perm, cfg = build()
    st = OracleGenericStack(config=cfg)
    st.SetState(nodes, allocs)
    st.SetJob(job)
    limit = st.SetNodes(list(perm))
    # the caller's loop (generic_sched.go:552-627, 773-792), every Select
    # answer kept: the plain Select's nil before a Preempt retry as well
    from nomad_amd.stack import SelectOptions
    res, nils, secs = [], [], []
    t0 = time.time()
    for i in range(CASE["count"]):
        t1 = time.perf_counter()
        r = st.SelectRaw(0)
        if r.row < 0:
            nils.append([i, r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted, r.new_offset])
            r = st.SelectRaw(0, SelectOptions(preempt=True))
        if r.row < 0:
            break
        st.Commit(0, r.row, r.preempted)
        secs.append(time.perf_counter() - t1)
        res.append(r)
    dt = time.time() - t0
    doc = {"case": CASE, "limit": limit, "oracle_seconds": dt, "placements": [record(r) for r in res],
           "plain_nils": nils}
    with gzip.open(OUT, "wt") as f:
        json.dump(doc, f, separators=(",", ":"))
    # where the oracle's time goes, placement by placement (bench.py's C5
    # cpu_baseline samples windows of this loop)
    prof = os.path.join(ROOT, "profiles", "r05", "c5_oracle_timing.json")
    os.makedirs(os.path.dirname(prof), exist_ok=True)
    with open(prof, "w") as f:
        json.dump({"case": CASE, "host": os.uname().nodename, "oracle_seconds": dt,
                   "evicting": [bool(r.preempted) for r in res], "seconds": secs}, f)
    print("wrote %s: %d placements, %d evicting, oracle %.1f s"
          % (OUT, len(res), sum(1 for r in res if r.preempted), dt))


if __name__ == "__main__":
    main()
