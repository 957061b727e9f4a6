"""Device-resident count loop over sparse options (k_ploop).

On a saturated cluster GenericScheduler.computePlacements runs one plain
Select per placement and retries it with Preempt=true when it is nil
(generic_sched.go:552-627, 773-792). The engine runs that whole loop in one
workgroup and re-evaluates only what a commit can change: the committed row,
and after an eviction every node whose Preempt outcome read the plan's
preemption counts (the max_parallel penalty, preemption.go:220-240). These
tests compare it placement by placement with the oracle, and with the
host-driven loop (PE_PLOOP=0) on the same engine.
"""
import os

import pytest

from nomad_amd import synth
from nomad_amd.structs import Allocation, SchedulerConfig
from oracle.oracle import OracleGenericStack
from tests.helpers import assert_same_placements, run_place

pytestmark = pytest.mark.gpu


def _engine(**kw):
    from nomad_amd.stack import GenericStack
    return GenericStack(**kw)


def _cpu_hogs(nodes, allocs, max_parallel):
    """A priority-20 CPU hog on every GPU node that already runs GPU work, sized
    so that the C5 ask (1000 MHz) only fits after the Preemptor also frees CPU
    (PreemptForTaskGroup after PreemptForDevice, rank.go:366-466)."""
    used = {}
    for a in allocs:
        used[a.node_id] = used.get(a.node_id, 0) + a.cpu_shares
    out = list(allocs)
    for k, nd in enumerate(nodes):
        if not nd.devices or nd.id not in used:
            continue
        hog = nd.cpu_shares - used[nd.id] - 500
        if hog > 0:
            out.append(Allocation(node_id=nd.id, job_id="hog-%d" % (k % 7), task_group="web", cpu_shares=hog,
                                  memory_mb=256, disk_mb=100, priority=20, max_parallel=max_parallel))
    return out


def _run_both(nodes, allocs, job, perm, cfg):
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm, config=cfg)
    _, _, re = run_place(_engine, nodes, allocs, job, perm, config=cfg)
    assert_same_placements(re, ro)
    assert [sorted(x.preempted) for x in re] == [sorted(x.preempted) for x in ro]
    assert [x.device_offers for x in re] == [x.device_offers for x in ro]
    return re, ro


@pytest.mark.parametrize("max_parallel", [None, 0])
def test_ploop_device_preemption(max_parallel):
    nodes, allocs = synth.cluster_c5(8000, seed=13, busy=0.99)
    if max_parallel is not None:
        for a in allocs:
            a.max_parallel = max_parallel
    job = synth.job_c5(300)
    perm = synth.shuffle(len(nodes), 5)
    re, _ = _run_both(nodes, allocs, job, perm, SchedulerConfig(preempt_service=True))
    assert sum(1 for x in re if x.preempted) > 100


@pytest.mark.parametrize("max_parallel", [1, 0])
def test_ploop_cpu_preemption_reads_plan_counts(max_parallel):
    """Evictions free GPUs and CPU; with max_parallel the distance penalty of
    every later eviction depends on the plan's preemption counts."""
    nodes, allocs = synth.cluster_c5(6000, seed=17, busy=0.99)
    allocs = _cpu_hogs(nodes, allocs, max_parallel)
    job = synth.job_c5(250)
    perm = synth.shuffle(len(nodes), 9)
    re, _ = _run_both(nodes, allocs, job, perm, SchedulerConfig(preempt_service=True))
    assert sum(1 for x in re if len(x.preempted) > 1) > 50


def test_ploop_matches_host_loop():
    nodes, allocs = synth.cluster_c5(20000, seed=21, busy=0.99)
    job = synth.job_c5(600)
    perm = synth.shuffle(len(nodes), 3)
    cfg = SchedulerConfig(preempt_service=True)
    _, _, dev = run_place(_engine, nodes, allocs, job, perm, config=cfg)
    os.environ["PE_PLOOP"] = "0"
    try:
        _, _, host = run_place(_engine, nodes, allocs, job, perm, config=cfg)
    finally:
        del os.environ["PE_PLOOP"]
    assert_same_placements(dev, host)
    assert [sorted(x.preempted) for x in dev] == [sorted(x.preempted) for x in host]


def test_ploop_cluster_exhausted():
    """More placements than the cluster can take even with eviction: the loop
    ends on a nil Preempt Select, as the caller's loop does (engine vs its
    host-driven loop, which the tests above pin to the oracle)."""
    nodes, allocs = synth.cluster_c5(5000, seed=23, busy=1.0)
    job = synth.job_c5(20000)
    perm = synth.shuffle(len(nodes), 4)
    cfg = SchedulerConfig(preempt_service=True)
    _, _, dev = run_place(_engine, nodes, allocs, job, perm, config=cfg)
    os.environ["PE_PLOOP"] = "0"
    try:
        _, _, host = run_place(_engine, nodes, allocs, job, perm, config=cfg)
    finally:
        del os.environ["PE_PLOOP"]
    assert dev[-1].row < 0 and 2000 < len(dev) < 20000
    assert_same_placements(dev, host)
    assert [sorted(x.preempted) for x in dev] == [sorted(x.preempted) for x in host]


@pytest.mark.parametrize("variant", ["max_parallel", "distinct_property", "job_counts"])
def test_ploop_skipped_plain_resolves_fail(variant, monkeypatch):
    """k_ploop skips a plain Select after a failed one whose placement left its
    row without a plain option. PE_PLOOP_CHECK_DEAD runs every
    skipped resolve anyway and fails the call (PE_EINTERNAL) if one finds a
    winner. Every GPU node is full (busy=1.0), so the plain Select stays dead
    across all the Preempt placements, with max_parallel penalties, a
    distinct_property constraint over a 40-rack meta key, or a job that
    already holds allocs (job-level collision counts) in play."""
    import random
    nodes, allocs = synth.cluster_c5(4000, seed=29, busy=1.0)
    rng = random.Random(3)
    for nd in nodes:
        nd.meta["rack"] = "r%02d" % rng.randrange(40)
        nd.compute_class()
    job = synth.job_c5(120)
    if variant == "max_parallel":
        for a in allocs:
            a.max_parallel = 1
    elif variant == "distinct_property":
        from nomad_amd.structs import Constraint
        job.task_groups[0].constraints.append(Constraint("${meta.rack}", "3", "distinct_property"))
    else:
        gpu = [nd for nd in nodes if nd.devices][:30]
        for nd in gpu:
            allocs.append(Allocation(node_id=nd.id, job_id=job.id, task_group="infer", cpu_shares=100,
                                     memory_mb=64, disk_mb=10, priority=80))
    perm = synth.shuffle(len(nodes), 6)
    monkeypatch.setenv("PE_PLOOP_CHECK_DEAD", "1")
    re, _ = _run_both(nodes, allocs, job, perm, SchedulerConfig(preempt_service=True))
    assert sum(1 for x in re if x.preempted) > 20


def test_ploop_near_the_lds_limit():
    """A list near the largest k_ploop takes (its codes fill the LDS the kernel's
    static use leaves, pe_ploop_max_n): the device loop against the host-driven
    loop of the same engine."""
    nodes, allocs = synth.cluster_c5(220000, seed=31, busy=0.999)
    job = synth.job_c5(200)
    perm = synth.shuffle(len(nodes), 6)
    cfg = SchedulerConfig(preempt_service=True)
    _, _, dev = run_place(_engine, nodes, allocs, job, perm, config=cfg)
    os.environ["PE_PLOOP"] = "0"
    try:
        _, _, host = run_place(_engine, nodes, allocs, job, perm, config=cfg)
    finally:
        del os.environ["PE_PLOOP"]
    assert_same_placements(dev, host)
    assert [sorted(x.preempted) for x in dev] == [sorted(x.preempted) for x in host]
    assert sum(1 for x in dev if x.preempted) > 10
