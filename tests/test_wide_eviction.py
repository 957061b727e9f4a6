"""Eviction past the narrow width (evict.inc): nodes holding
more than 32 allocs, priority groups longer than 12 (Go 1.16's sort.Slice in
full: quickSort_func, the ninther past 40 elements, heapSort past the depth
limit), more than PE_MAX_PREEMPT preempted allocs (pe_preempted_of) and
ProposedAllocs lists longer than 64 (a launch flags the node and the engine
reruns it wider). PreemptForTaskGroup walks every alloc of the node
(scheduler/preemption.go:146-267) and sorts groups of any length
(preemption.go:663-699); rank.go:511-513 has no cap on PreemptedAllocs.
Engine vs oracle, placement by placement, preempted sets included.
"""
import numpy as np
import pytest

from nomad_amd import synth
from nomad_amd.structs import Allocation, DeviceGroup, Job, RequestedDevice, SchedulerConfig, Task, TaskGroup
from oracle.oracle import OracleGenericStack
from tests.helpers import assert_same_placements, run_place

pytestmark = pytest.mark.gpu

GPU_ATTRS = {"memory": (80, "GiB")}


def _engine(**kw):
    from nomad_amd.stack import GenericStack
    return GenericStack(**kw)


def wide_cluster(n_nodes, per_node, seed, devices=False, tie_every=0):
    """Nodes packed with `per_node` small low-priority allocs each (priorities
    20 / 30 / 40 from several jobs, varied sizes so the distance sort has work
    to do; with `tie_every` every k-th alloc repeats a size so the unstable
    sort's treatment of equal keys shows)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes, allocs = [], []
    for k in range(n_nodes):
        nd = synth.mock_node("wide-%04d" % k)
        nd.name = "wide-%04d" % k
        nd.cpu_shares = 64000
        nd.memory_mb = 131072
        nd.disk_mb = 400 * 1024
        if devices:
            nd.devices = [DeviceGroup("nvidia", "gpu", "h100", 64, dict(GPU_ATTRS))]
        nd.compute_class()
        nodes.append(nd)
        used_c = used_m = 0
        for i in range(per_node):
            if tie_every and i % tie_every == 0:
                c, m = 400, 800
            else:
                c = int(rng.integers(100, 900))
                m = int(rng.integers(200, 1800))
            prio = int(rng.choice([20, 30, 40]))
            a = Allocation(node_id=nd.id, job_id="bg-%d" % (i % 9), task_group="w%d" % (i % 3), cpu_shares=c,
                           memory_mb=m, disk_mb=100, priority=prio, max_parallel=(i % 4))
            if devices and i < 64:
                a.devices = [(0, 1)]
            allocs.append(a)
            used_c += c
            used_m += m
        # fill the node so that an ask needs evictions
        rest_c = nd.cpu_shares - nd.reserved_cpu - used_c - 50
        rest_m = nd.memory_mb - nd.reserved_memory_mb - used_m - 50
        if rest_c > 0 and rest_m > 0:
            allocs.append(Allocation(node_id=nd.id, job_id="filler", task_group="f", cpu_shares=rest_c,
                                     memory_mb=rest_m, disk_mb=100, priority=95))
    return nodes, allocs


def big_ask_job(count, cpu, mem, gpus=0):
    devs = [RequestedDevice("nvidia/gpu", gpus)] if gpus else []
    return Job(id="big", priority=100, task_groups=[TaskGroup(name="big", count=count, ephemeral_disk_mb=10, tasks=[
        Task(name="t", driver="exec", cpu=cpu, memory_mb=mem, devices=devs)])])


def _both(nodes, allocs, job, perm):
    cfg = SchedulerConfig(preempt_service=True)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm, config=cfg)
    _, _, re = run_place(_engine, nodes, allocs, job, perm, config=cfg)
    assert_same_placements(re, ro)
    assert [sorted(x.preempted) for x in re] == [sorted(x.preempted) for x in ro]
    assert [x.device_offers for x in re] == [x.device_offers for x in ro]
    return re


@pytest.mark.parametrize("per_node", [40, 64, 128, 250])
def test_task_group_preemption_on_wide_nodes(per_node):
    # each placement frees ~10k MHz of 100-900 MHz allocs: long priority
    # groups, > 16 preempted allocs per placement
    nodes, allocs = wide_cluster(24, per_node, seed=per_node)
    job = big_ask_job(20, 9000, 2000)
    re = _both(nodes, allocs, job, synth.shuffle(len(nodes), 3))
    assert sum(1 for x in re if x.row >= 0) >= 10
    assert max(len(x.preempted) for x in re) > 16


@pytest.mark.parametrize("tie_every", [2, 3])
def test_equal_distance_ties_in_long_groups(tie_every):
    """Equal basicResourceDistance keys: the order the unstable sort leaves
    them in decides which allocs filterSuperset keeps."""
    nodes, allocs = wide_cluster(12, 96, seed=7 + tie_every, tie_every=tie_every)
    job = big_ask_job(10, 6000, 1000)
    _both(nodes, allocs, job, synth.shuffle(len(nodes), 4))


def test_device_preemption_on_wide_nodes():
    # 64 single-GPU allocs per node: PreemptForDevice over long lists
    nodes, allocs = wide_cluster(16, 100, seed=11, devices=True)
    job = big_ask_job(12, 500, 500, gpus=20)
    re = _both(nodes, allocs, job, synth.shuffle(len(nodes), 5))
    assert max(len(x.preempted) for x in re) >= 20


def test_mixed_widths_one_wide_node():
    """One node past 32 allocs in an otherwise narrow cluster: the whole
    snapshot evaluates at the wide width (it used to refuse every Preempt
    Select of the cluster)."""
    nodes, allocs = synth.cluster_c5(3000, seed=31, busy=0.99)
    wn, wa = wide_cluster(1, 80, seed=2, devices=True)
    nodes = nodes + wn
    allocs = allocs + wa
    job = synth.job_c5(200)
    _both(nodes, allocs, job, synth.shuffle(len(nodes), 8))


def test_proposed_allocs_outgrow_the_narrow_width():
    """30 state allocs (narrow snapshot) plus > 34 plan placements of the job on
    one node: ProposedAllocs passes 64 entries, the narrow launch flags the
    node and the Select reruns wide."""
    nd = synth.mock_node("solo")
    nd.name = "solo"
    nd.cpu_shares, nd.memory_mb = 12000, 65536
    nd.compute_class()
    allocs = [Allocation(node_id=nd.id, job_id="low-%d" % (i % 3), task_group="w", cpu_shares=180, memory_mb=256,
                         disk_mb=10, priority=20) for i in range(30)]
    job = big_ask_job(90, 150, 64)
    _both([nd], allocs, job, [0])


def test_select_commit_protocol_with_long_preempted_lists():
    """The caller's Select(Preempt) -> Commit(row, PreemptedAllocs) with
    lists past PE_MAX_PREEMPT: the stack wrapper reads the full list with
    pe_preempted_of and commits it."""
    from nomad_amd.stack import SelectOptions
    nodes, allocs = wide_cluster(8, 128, seed=5)
    job = big_ask_job(6, 9000, 2000)
    cfg = SchedulerConfig(preempt_service=True)
    out = []
    for cls in (OracleGenericStack, _engine):
        st = cls(config=cfg)
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(list(synth.shuffle(len(nodes), 6)))
        res = []
        for _ in range(6):
            r = st.Select(0)
            if r is None:
                r = st.Select(0, SelectOptions(preempt=True))
            if r is None:
                break
            st.Commit(0, r.row, r.preempted)
            res.append((r.row, r.final_score, sorted(r.preempted)))
        out.append(res)
    assert out[0] == out[1]
    assert max(len(x[2]) for x in out[0]) > 16


def dense_cluster(n_nodes, per_node, seed):
    """Nodes of `per_node` (> 256) small low-priority allocs, sized so that the
    node holds them all: the widest eviction width (W = 32, 1024 allocs)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes, allocs = [], []
    for k in range(n_nodes):
        nd = synth.mock_node("dense-%04d" % k)
        nd.name = "dense-%04d" % k
        nd.cpu_shares = per_node * 520 + 2000
        nd.memory_mb = per_node * 1050 + 4096
        nd.disk_mb = per_node * 110 + 8192
        nd.compute_class()
        nodes.append(nd)
        for i in range(per_node):
            allocs.append(Allocation(node_id=nd.id, job_id="bg-%d" % (i % 11), task_group="w%d" % (i % 3),
                                     cpu_shares=int(rng.integers(100, 900)), memory_mb=int(rng.integers(200, 1800)),
                                     disk_mb=100, priority=int(rng.choice([20, 30, 40])), max_parallel=(i % 4)))
    return nodes, allocs


@pytest.mark.parametrize("per_node", [300, 600])
def test_preemption_past_256_allocs(per_node):
    """Nodes of 300 and 600 allocs: PreemptForTaskGroup over the whole list
    at W = 32 (masks of 32 words, index lists of 1024 / 2048 entries in the
    lane's scratch); the count loop takes the per-Select path past k_ploop's
    width. Placement by placement equal to the oracle."""
    nodes, allocs = dense_cluster(6, per_node, seed=per_node)
    job = big_ask_job(8, 30000, 8000)
    re = _both(nodes, allocs, job, synth.shuffle(len(nodes), 7))
    assert sum(1 for x in re if x.row >= 0) >= 4
    assert max(len(x.preempted) for x in re) > 16


def test_proposed_allocs_past_512():
    """250 state allocs (a W = 8 snapshot) plus more than 262 plan placements
    of the job on the node: ProposedAllocs passes 512 entries and the evicting
    Selects rerun at W = 32."""
    nd = synth.mock_node("solo")
    nd.name = "solo"
    nd.cpu_shares, nd.memory_mb, nd.disk_mb = 100000, 1 << 20, 1 << 20
    nd.compute_class()
    allocs = [Allocation(node_id=nd.id, job_id="low-%d" % (i % 3), task_group="w", cpu_shares=200, memory_mb=256,
                         disk_mb=10, priority=20) for i in range(250)]
    job = big_ask_job(420, 150, 64)
    re = _both([nd], allocs, job, [0])
    assert sum(1 for x in re if x.row >= 0) > 340
    assert any(x.preempted for x in re)
