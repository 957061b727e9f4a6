"""One engine handle over several GPUs (pe_config.device_count / device_ids).

SURVEY.md §8(b) asks for a handle a single Go process can own across GPUs
(device count and ids; the handle owns the communicators). The handle keeps
replicas of the snapshot, job and plan on the other devices; full-pass count
loops (C3-shaped task groups: affinities / spreads, limit MaxInt32) and the
SystemScheduler batch split their rows over the replicas and exchange the
per-placement LimitIterator/MaxScoreIterator records (ncclAllGather over
communicators from ncclCommInitAll). Here every id names GPU 0, the loopback
mode: N virtual shards each sweep their row range into their own slice of
their gather buffer, the slices are copied between replicas, and every
replica's k_sweep_step merges N x blocks records and commits the same winner,
exactly the layout the RCCL path uses (VERDICT r02 missing 4 / weak 3).
Results must equal a single-device handle and the oracle, for N = 2, 3, 8.
"""
import dataclasses

import numpy as np
import pytest

from nomad_amd import synth
from nomad_amd.structs import Allocation, Constraint, Task, TaskGroup
from oracle.oracle import OracleGenericStack, OracleSystemStack
from tests.helpers import assert_same_placements, run_place

pytestmark = pytest.mark.gpu


def generic(n_dev):
    from nomad_amd.stack import GenericStack
    return GenericStack(devices=[0] * n_dev) if n_dev > 1 else GenericStack()


def system(n_dev):
    from nomad_amd.stack import SystemStack
    return SystemStack(devices=[0] * n_dev) if n_dev > 1 else SystemStack()


@pytest.fixture(scope="module")
def c3_case():
    nodes, allocs = synth.cluster_c3(3000, seed=7)
    job = synth.job_c3(300)
    perm = synth.shuffle(len(nodes), 21)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm)
    return nodes, allocs, job, perm, ro


@pytest.mark.parametrize("n_dev", [2, 3, 8])
def test_full_pass_loop_split_over_devices(c3_case, n_dev):
    nodes, allocs, job, perm, ro = c3_case
    st, _, re_ = run_place(lambda: generic(n_dev), nodes, allocs, job, perm)
    import ctypes as C
    assert st._lib.pe_device_count(C.c_void_p(st._h)) == n_dev
    assert_same_placements(re_, ro)


@pytest.mark.parametrize("n_dev", [2, 3])
def test_replicas_follow_the_plan(n_dev):
    """Placements made on the root alone (a windowed group through Select /
    Commit, plan stops) are replayed into the replicas before the split loop
    of the full-pass group, over two evaluations on one handle."""
    nodes, allocs = synth.cluster_c3(2000, seed=5)
    rng = np.random.Generator(np.random.PCG64(9))
    for k in rng.choice(len(nodes), size=60, replace=False):
        allocs.append(Allocation(node_id=nodes[int(k)].id, job_id="svc-c3", task_group="web", cpu_shares=300,
                                 memory_mb=128, disk_mb=100))
    base = synth.job_c3(120)
    win = TaskGroup(name="batchy", count=80, ephemeral_disk_mb=150,
                    constraints=[Constraint("${attr.kernel.name}", "linux", "=")],
                    tasks=[Task(name="b", driver="exec", cpu=400, memory_mb=300)])
    job = dataclasses.replace(base, task_groups=[win, base.task_groups[0]])
    e, o = generic(n_dev), OracleGenericStack()
    for st in (e, o):
        st.SetState(nodes, allocs)
    own = [i for i, a in enumerate(allocs) if a.job_id == "svc-c3"]
    for ev in range(2):
        for st in (e, o):
            if ev:
                st.ResetPlan()
            st.SetJob(job)
            st.SetNodes(list(synth.shuffle(len(nodes), 30 + ev)))
            st.StopAllocs(own[10 * ev:10 * ev + 10])
        for _ in range(40):
            a, b = o.SelectRaw(0), e.SelectRaw(0)
            assert_same_placements([b], [a])
            if a.row < 0:
                break
            o.Commit(0, a.row)
            e.Commit(0, b.row)
        assert_same_placements(e.Place(1, 120), o.Place(1, 120))
        assert_same_placements(e.Place(1, 40), o.Place(1, 40))   # the replicas kept the plan


@pytest.mark.parametrize("n_dev", [2, 8])
def test_system_batch_split_over_devices(n_dev):
    nodes, allocs = synth.cluster_c4(20000, seed=11)
    job = synth.mock_system_job()
    rows = np.random.Generator(np.random.PCG64(4)).permutation(len(nodes)).astype(np.uint32)
    o = OracleSystemStack()
    o.SetState(nodes, allocs)
    o.SetJob(job)
    o.SetNodes(rows)
    so, to, po = o.SystemPlace(0)
    e = system(n_dev)
    e.SetState(nodes, allocs)
    e.SetJob(job)
    e.SetNodes(rows)
    se, te, pe_ = e.SystemPlace(0)
    assert pe_ == po and np.array_equal(te, to) and np.array_equal(se[te == 0], so[to == 0])
    # a second pass over the same list: every replica must hold every placement
    o.SetNodes(rows)
    e.SetNodes(rows)
    so2, to2, po2 = o.SystemPlace(0)
    se2, te2, pe2 = e.SystemPlace(0)
    assert pe2 == po2 and np.array_equal(te2, to2)
