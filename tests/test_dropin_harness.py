"""The C caller harness (tools/libdropin.so) that bench.py times: on the CPU
oracle, its Select -> Commit loop must place exactly what the oracle's own
count loop places (CPU); on the GPU, the engine driven by the same loop must
equal the oracle driven by it."""
import numpy as np
import pytest

from nomad_amd import synth
from nomad_amd.structs import SchedulerConfig
from oracle.oracle import OracleGenericStack
from tools import dropin


def test_harness_matches_oracle_place():
    nodes, allocs = synth.cluster_c2(600, seed=42)
    job = synth.job_c2(120)
    orders = np.stack([synth.shuffle(600, 3), synth.shuffle(600, 4)])
    st = OracleGenericStack()
    st.SetState(nodes, allocs)
    placed, evals, selects, secs, rows = dropin.run(st, job, orders, 120)
    assert evals == 2 and placed == 240 and selects == 240
    ref = OracleGenericStack()
    ref.SetState(nodes, allocs)
    ref.SetJob(job)
    ref.SetNodes(orders[1])
    want = ref.PlaceArrays(0, 120)[0]
    assert list(rows) == list(want)


def test_harness_preempt_retry_on_oracle():
    nodes, allocs = synth.cluster_c5(300, seed=5, busy=0.95)
    job = synth.job_c5(60)
    cfg = SchedulerConfig(preempt_service=True)
    st = OracleGenericStack(config=cfg)
    st.SetState(nodes, allocs)
    order = synth.shuffle(300, 77)
    placed, evals, selects, _, rows = dropin.run(st, job, order, 60, preempt=True)
    ref = OracleGenericStack(config=cfg)
    ref.SetState(nodes, allocs)
    ref.SetJob(job)
    ref.SetNodes(order)
    res = ref.Place(0, 60)          # pe_place retries with Preempt itself
    want = [r.row for r in res if r.row >= 0]
    assert list(rows[:placed]) == want
    assert selects > placed         # some Selects were nil and retried with Preempt


@pytest.mark.gpu
def test_engine_through_harness_equals_oracle():
    from nomad_amd.stack import GenericStack
    nodes, allocs = synth.cluster_c2(5000, seed=42)
    job = synth.job_c2(1000)
    orders = np.stack([synth.shuffle(5000, s) for s in (11, 12, 13)])
    got = []
    for st in (GenericStack(), OracleGenericStack()):
        st.SetState(nodes, allocs)
        placed, evals, _, _, rows = dropin.run(st, job, orders, 1000)
        got.append((placed, evals, list(rows)))
    assert got[0] == got[1]
