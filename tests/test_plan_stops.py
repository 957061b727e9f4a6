"""Plan stops (Plan.AppendStoppedAlloc, structs.go:10628-10660, and PopUpdate,
:10691-10702): a stopped snapshot alloc leaves its node's proposed state
(EvalContext.ProposedAllocs, context.go:120-157) and is counted as cleared by
the property sets (propertyset.go:159-209). They come from computeJobAllocs
(generic_sched.go:382), destructive updates (:546, popped at :644 when the
replacement fails), inplaceUpdate / genericAllocUpdateFn (util.go:749-756,
1037-1043) and the SystemScheduler (scheduler_system.go:230-241).

CPU tests pin the oracle's NodeUpdate model to the reference semantics; GPU
tests compare the engine with the oracle Select by Select."""
import numpy as np
import pytest

from nomad_amd import synth
from nomad_amd.structs import Allocation, Constraint, Job, SchedulerConfig, Task, TaskGroup
from oracle.oracle import OracleGenericStack, OracleSystemStack


def _key(r):
    if r is None:
        return None
    return (r.row, r.final_score, tuple(r.scores), r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted,
            r.new_offset, tuple(r.preempted), tuple(r.device_offers))


def _loop(st, count, tg=0, preempt=False):
    from nomad_amd.stack import SelectOptions
    out = []
    for _ in range(count):
        opt = st.Select(tg)
        if opt is None and preempt:
            opt = st.Select(tg, SelectOptions(preempt=True))
        out.append(_key(opt))
        if opt is None:
            break
        st.Commit(tg, opt.row, opt.preempted)
    return out


def _job_with_own_allocs(n, own, seed, spread=False, distinct=None):
    """A C2-shaped cluster where job 'svc-c2' (an older version) already holds
    `own` allocs on random nodes, plus the foreign ones."""
    nodes, allocs = synth.cluster_c2(n, seed=seed)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    for k in rng.choice(n, size=own, replace=False):
        allocs.append(Allocation(node_id=nodes[int(k)].id, job_id="svc-c2", task_group="web",
                                 cpu_shares=500, memory_mb=256, disk_mb=150, priority=50))
    job = synth.job_c2(own)
    job.version = 7
    if spread:
        from nomad_amd.structs import Spread, SpreadTarget
        job.task_groups[0].spreads = [Spread("${node.class}", 60, [SpreadTarget("class-1", 40),
                                                                 SpreadTarget("class-2", 30)])]
    if distinct:
        job.task_groups[0].constraints = [Constraint("${node.class}", str(distinct), "distinct_property")]
    own_idx = [i for i, a in enumerate(allocs) if a.job_id == "svc-c2"]
    return nodes, allocs, job, own_idx


# ---- oracle (CPU) ---------------------------------------------------------------

def test_oracle_stop_frees_the_node():
    # one node, filled by one alloc: infeasible until the alloc is stopped,
    # feasible again after, and PopUpdate brings the alloc back
    nodes, _ = synth.cluster_c1(1, seed=3)
    nd = nodes[0]
    big = Allocation(node_id=nd.id, job_id="other", task_group="tg", cpu_shares=nd.cpu_shares - 100 - 100,
                     memory_mb=nd.memory_mb - 256 - 100, disk_mb=100)
    job = synth.mock_job(count=1)
    st = OracleGenericStack()
    st.SetState(nodes, [big])
    st.SetJob(job)
    st.SetNodes([0])
    assert st.Select(0) is None
    st.StopAllocs([0])
    opt = st.Select(0)
    assert opt is not None and opt.row == 0
    st.PopUpdate(0)
    assert st.Select(0) is None


def test_oracle_pop_update_only_drops_the_last_entry():
    nodes, _ = synth.cluster_c1(1, seed=4)
    nd = nodes[0]
    a = [Allocation(node_id=nd.id, job_id="other", task_group="tg", cpu_shares=1800, memory_mb=3000, disk_mb=100)
         for _ in range(2)]
    job = synth.mock_job(count=1)
    st = OracleGenericStack()
    st.SetState(nodes, a)
    st.SetJob(job)
    st.SetNodes([0])
    assert st.Select(0) is None          # 1800 + 1800 + the ask exceed the node's 3900 cpu
    st.StopAllocs([0, 1])
    st.PopUpdate(0)                      # not the last NodeUpdate entry of the node: no effect
    assert st.Select(0) is not None
    st.PopUpdate(1)                      # alloc 1 is back; alloc 0 stays stopped
    assert st.Select(0) is not None
    st.PopUpdate(0)
    assert st.Select(0) is None


def test_oracle_stopped_own_allocs_leave_the_collision_count():
    # JobAntiAffinity (rank.go:564-597) counts ProposedAllocs of the job: a
    # stopped alloc of the job no longer collides
    nodes, allocs, job, own = _job_with_own_allocs(40, 10, seed=5)
    st = OracleGenericStack()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    rows_with_own = sorted({st.row(allocs[i].node_id) for i in own})
    st.SetNodes(rows_with_own[:1])
    before = st.Select(0)
    st.StopAllocs([i for i in own if st.row(allocs[i].node_id) == rows_with_own[0]])
    after = st.Select(0)
    assert before is not None and after is not None
    assert len(after.scores) < len(before.scores)     # the anti-affinity score is gone


# ---- engine vs oracle (GPU) -----------------------------------------------------

def _both(nodes, allocs, job, perm, prep, count, config=None, preempt=False, system=False):
    from nomad_amd.stack import GenericStack, SystemStack
    res = []
    if system:
        pairs = (SystemStack(config=config), OracleSystemStack(config=config))
    else:
        pairs = (GenericStack(config=config), OracleGenericStack(config=config))
    for st in pairs:
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
        prep(st)
        if system:
            sc, status, placed = st.SystemPlace(0)
            res.append((list(np.asarray(status)), [float(x) for x in np.asarray(sc)], placed))
        else:
            res.append(_loop(st, count, preempt=preempt))
    return res


@pytest.mark.gpu
def test_stops_of_foreign_allocs_count_loop():
    nodes, allocs = synth.cluster_c2(3000, seed=61)
    job = synth.job_c2(600)
    rng = np.random.Generator(np.random.PCG64(3))
    stop = sorted(int(x) for x in rng.choice(len(allocs), size=len(allocs) // 3, replace=False))
    a, b = _both(nodes, allocs, job, synth.shuffle(3000, 7), lambda st: st.StopAllocs(stop), 600)
    assert a == b


@pytest.mark.gpu
def test_destructive_update_stops_own_allocs():
    nodes, allocs, job, own = _job_with_own_allocs(2500, 400, seed=62)
    stop = own[::2]
    a, b = _both(nodes, allocs, job, synth.shuffle(2500, 8), lambda st: st.StopAllocs(stop), 200)
    assert a == b


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["spread", "distinct"])
def test_cleared_property_values(kind):
    nodes, allocs, job, own = _job_with_own_allocs(1500, 120, seed=63, spread=kind == "spread",
                                                   distinct=40 if kind == "distinct" else None)
    stop = own[:80]
    a, b = _both(nodes, allocs, job, synth.shuffle(1500, 9), lambda st: st.StopAllocs(stop), 150)
    assert a == b


@pytest.mark.gpu
def test_inplace_update_stop_select_pop():
    # inplaceUpdate (util.go:743-760): stop the alloc, Select on its node only,
    # PopUpdate, then the updated alloc replaces the old one (commit)
    nodes, allocs, job, own = _job_with_own_allocs(800, 60, seed=64)
    from nomad_amd.stack import GenericStack
    seqs = []
    for st in (GenericStack(), OracleGenericStack()):
        st.SetState(nodes, allocs)
        st.SetJob(job)
        seq = []
        for i in own[:40]:
            row = st.row(allocs[i].node_id)
            st.StopAllocs([i])
            st.SetNodes([row])
            opt = st.Select(0)
            seq.append(_key(opt))
            st.PopUpdate(i)
            if opt is not None:
                st.StopAllocs([i])        # the in-place alloc replaces the old one (same ID)
                st.Commit(0, opt.row)
        st.SetNodes(synth.shuffle(800, 10))
        seq += _loop(st, 30)
        seqs.append(seq)
    assert seqs[0] == seqs[1]


@pytest.mark.gpu
def test_stops_with_devices_and_preemption():
    nodes, allocs = synth.cluster_c5(900, seed=65, busy=0.9)
    job = synth.job_c5(100)
    stop = list(range(0, len(allocs), 5))
    cfg = SchedulerConfig(preempt_service=True)
    a, b = _both(nodes, allocs, job, synth.shuffle(900, 11), lambda st: st.StopAllocs(stop), 100, config=cfg,
                 preempt=True)
    assert a == b


@pytest.mark.gpu
def test_system_scheduler_stops():
    nodes, allocs = synth.cluster_c4(3000, seed=66)
    job = synth.mock_system_job()
    stop = list(range(0, len(allocs), 3))
    a, b = _both(nodes, allocs, job, np.arange(3000, dtype=np.uint32), lambda st: st.StopAllocs(stop), 0,
                 system=True)
    assert a[0] == b[0] and a[2] == b[2]
    np.testing.assert_array_equal(np.asarray(a[1]), np.asarray(b[1]))
