"""Reserved cores (BinPackIterator, rank.go:437-466; AllocsFit core checks,
funcs.go:148-180 and structs.go:3891-3906).

A task asking `cores` takes the lowest free cores of the node's
ReservableCpuCores (cores held by the node's proposed allocs and by earlier
tasks are not free), and holds SharesPerCore x cores CpuShares instead of its
CPU ask. AllocsFit then fails with "cores" when the chosen cores are outside
ReservableCpuCores - ReservedCpuCores (a reference quirk kept on both sides).
Engine vs oracle placement by placement, reserved cores included, over the
windowed chain, the full-pass loops, the caller's Select / Commit protocol,
the SystemStack and plan stops; the oracle is pinned by the reference's
TestBinPackIterator_ReservedCores KAT (tests/test_reference_kats.py).
"""
import numpy as np
import pytest

from nomad_amd import synth
from nomad_amd.structs import Affinity, Allocation, Job, SchedulerConfig, Task, TaskGroup
from oracle.oracle import OracleGenericStack, OracleSystemStack
from tests.helpers import assert_same_placements, run_place


def cluster_cores(n, seed, allocs_frac=0.5):
    rng = np.random.Generator(np.random.PCG64(seed))
    ids = sorted(synth.uuids(n, seed))
    nodes, allocs = [], []
    for k, nid in enumerate(ids):
        nd = synth.mock_node(nid)
        nd.name = "node-%05d" % k
        total = int(rng.choice([4, 8, 16, 32, 64, 128]))
        nd.total_cores = total
        nd.cpu_shares = total * int(rng.choice([1000, 2000, 2500]))
        nd.memory_mb = int(rng.choice([8192, 16384, 65536]))
        start = int(rng.integers(0, 2))                        # core 0 sometimes kept by the OS
        nd.reservable_cores = list(range(start, total))
        if rng.random() < 0.2:
            nd.reserved_cores = [start]                        # ReservedCpuCores (AllocsFit quirk)
        nd.compute_class()
        nodes.append(nd)
        if rng.random() < allocs_frac:
            free = [c for c in nd.reservable_cores if c not in nd.reserved_cores]
            take = list(rng.choice(free, size=min(len(free), int(rng.integers(1, 1 + len(free)))), replace=False))
            spc = nd.cpu_shares // total
            allocs.append(Allocation(node_id=nid, job_id="other-%d" % (k % 5), task_group="web",
                                     cpu_shares=spc * len(take), memory_mb=512, disk_mb=100, priority=50,
                                     reserved_cores=sorted(int(c) for c in take)))
    return nodes, allocs


def cores_job(count, cores=2, affinity=False, job_id="cores-job"):
    tg = TaskGroup(name="pinned", count=count, ephemeral_disk_mb=100, tasks=[
        Task(name="main", driver="exec", cpu=0, memory_mb=256, cores=cores),
        Task(name="side", driver="exec", cpu=100, memory_mb=64)])
    if affinity:
        tg.affinities = [Affinity("${node.unique.name}", "node-0", ">=", 40)]
    return Job(id=job_id, task_groups=[tg])


def _engine(**kw):
    from nomad_amd.stack import GenericStack
    return GenericStack(**kw)


def _same(re, ro):
    assert_same_placements(re, ro)
    assert [x.reserved_cores for x in re] == [x.reserved_cores for x in ro]


def test_cores_oracle_takes_lowest_free():
    nodes, allocs = cluster_cores(50, seed=3)
    job = cores_job(30, cores=3)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, synth.shuffle(len(nodes), 1))
    held = {}
    for a in allocs:
        held.setdefault(a.node_id, set()).update(a.reserved_cores)
    for r in ro:
        if r.row < 0:
            continue
        nd = nodes[r.row]
        free = [c for c in nd.reservable_cores if c not in held.get(nd.id, set())]
        assert r.reserved_cores == free[:3]
        held.setdefault(nd.id, set()).update(r.reserved_cores)


@pytest.mark.gpu
@pytest.mark.parametrize("n,count,affinity", [(600, 400, False), (3000, 300, True), (12000, 200, True)])
def test_cores_count_loop(n, count, affinity):
    nodes, allocs = cluster_cores(n, seed=n)
    job = cores_job(count, cores=2, affinity=affinity)
    perm = synth.shuffle(len(nodes), 7)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm)
    _, _, re = run_place(_engine, nodes, allocs, job, perm)
    _same(re, ro)
    assert any(x.reserved_cores for x in re)


@pytest.mark.gpu
def test_cores_select_commit_protocol_and_metrics():
    nodes, allocs = cluster_cores(800, seed=11)
    job = cores_job(150, cores=4)
    perm = synth.shuffle(len(nodes), 2)
    sts = []
    for cls in (OracleGenericStack, _engine):
        st = cls()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
        st.EnableMetrics(True)
        sts.append(st)
    exhausted_cores = 0
    for _ in range(150):
        ro, re = (st.SelectRaw(0) for st in sts)
        _same([re], [ro])
        mo, me = (st.LastMetrics() for st in sts)
        assert me == mo
        exhausted_cores += mo.get("DimensionExhausted", {}).get("cores", 0)
        if ro.row < 0:
            break
        for st in sts:
            st.Commit(0, ro.row)
    assert exhausted_cores > 0


@pytest.mark.gpu
def test_cores_system_stack():
    from nomad_amd.stack import SystemStack
    nodes, allocs = cluster_cores(2000, seed=5)
    job = cores_job(1, cores=8, job_id="sys-cores")
    job.type = 2
    out = []
    for cls in (OracleSystemStack, SystemStack):
        st = cls()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(list(range(len(nodes))))
        out.append(st.SystemPlace(0))
    (so, to, po), (se, te, pe) = out
    assert po == pe and (to == te).all()
    m = to == 0
    assert (so[m] == se[m]).all()


@pytest.mark.gpu
def test_cores_plan_stop_frees_cores():
    nodes, allocs = cluster_cores(200, seed=9, allocs_frac=1.0)
    job = cores_job(5, cores=1)
    plain = {nd.id for nd in nodes if not nd.reserved_cores}   # no ReservedCpuCores quirk on the node
    victim = max((i for i in range(len(allocs)) if allocs[i].node_id in plain),
                 key=lambda i: len(allocs[i].reserved_cores))
    row = next(i for i, nd in enumerate(nodes) if nd.id == allocs[victim].node_id)
    res = []
    for cls in (OracleGenericStack, _engine):
        st = cls()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes([row])
        before = st.SelectRaw(0)
        st.StopAllocs([victim])
        after = st.SelectRaw(0)
        st.Commit(0, after.row)
        again = st.SelectRaw(0)
        res.append((before, after, again))
    for x, y in zip(*res):
        _same([y], [x])
    assert res[0][1].row == row and res[0][1].reserved_cores[0] <= min(allocs[victim].reserved_cores)


@pytest.mark.gpu
def test_cores_fallbacks_are_explicit():
    from nomad_amd.stack import Unsupported
    nodes, allocs = cluster_cores(100, seed=4, allocs_frac=1.0)
    # overlapping alloc core sets fail every AllocsFit on the node: host path
    a = allocs[0]
    allocs.append(Allocation(node_id=a.node_id, job_id="dup", task_group="web", cpu_shares=1, memory_mb=1,
                             reserved_cores=list(a.reserved_cores[:1])))
    st = _engine()
    st.SetState(nodes, allocs)
    st.SetJob(cores_job(1))
    st.SetNodes(list(range(len(nodes))))
    with pytest.raises(Unsupported):
        st.SelectRaw(0)
    # cores with preemption (the reference's "TODO preemption")
    nodes, allocs = cluster_cores(100, seed=4)
    st = _engine(config=SchedulerConfig(preempt_service=True))
    st.SetState(nodes, allocs)
    st.SetJob(cores_job(1))
    st.SetNodes(list(range(len(nodes))))
    from nomad_amd.stack import SelectOptions
    with pytest.raises(Unsupported):
        st.SelectRaw(0, SelectOptions(preempt=True))


def _evicting_cores_cluster(n, seed):
    """Every node full: one priority-20 alloc holds 7000 MB and reserved cores
    1-6 of 8, so a 4096 MB ask evicts it and a cores=4 ask fits only where it
    is gone (cores 0 and 7 stay free otherwise)."""
    ids = sorted(synth.uuids(n, seed))
    nodes, allocs = [], []
    for k, nid in enumerate(ids):
        nd = synth.mock_node(nid)
        nd.name = "node-%05d" % k
        nd.total_cores = 8
        nd.cpu_shares = 8000
        nd.memory_mb = 8192
        nd.reservable_cores = list(range(8))
        nd.compute_class()
        nodes.append(nd)
        allocs.append(Allocation(node_id=nid, job_id="batch-%d" % (k % 7), task_group="train",
                                 cpu_shares=6000, memory_mb=7000, disk_mb=100, priority=20,
                                 reserved_cores=[1, 2, 3, 4, 5, 6]))
    return nodes, allocs


@pytest.mark.gpu
@pytest.mark.parametrize("via_view", [True, False])
def test_rolled_back_evictions_keep_their_cores(via_view):
    """A speculative run whose placements evict allocs holding reserved cores,
    rolled back by a deviating commit: the unconfirmed evictions'
    cores are held again on the device and in the host mirror, so the cores
    asks of the next task group see exactly the oracle's used sets."""
    from nomad_amd.stack import GenericStack
    from tests.test_spec_view import CCaller, ViewAnswers, protocol_answers
    from tests.test_dropin import assert_equal_runs
    nodes, allocs = _evicting_cores_cluster(300, seed=12)
    job = Job(id="evictor", priority=80, task_groups=[
        TaskGroup(name="big", count=40, ephemeral_disk_mb=100,
                  tasks=[Task(name="m", driver="exec", cpu=500, memory_mb=4096)]),
        TaskGroup(name="pinned", count=30, ephemeral_disk_mb=100,
                  tasks=[Task(name="p", driver="exec", cpu=0, memory_mb=256, cores=4)])])
    perm = synth.shuffle(len(nodes), 4)
    cfg = SchedulerConfig(preempt_service=True)
    eng, ora = GenericStack(config=cfg), OracleGenericStack(config=cfg)
    for st in (eng, ora):
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
    dev = lambda i, row: (int(perm[(i * 11) % len(perm)]) if i % 7 == 3 else None)
    ce = ViewAnswers(eng) if via_view else CCaller(eng)
    a = protocol_answers(ce, 40, deviate=dev, tg=0) + protocol_answers(ce, 30, tg=1)
    b = protocol_answers(CCaller(ora), 40, deviate=dev, tg=0) + protocol_answers(CCaller(ora), 30, tg=1)
    assert_equal_runs(a, b)
    assert eng.SpeculationStats()[2] >= 3   # rollbacks happened
    assert sum(1 for x in b if x[0] != "nil" and x[7]) >= 40, "too few evicting placements"
