"""distinct_property: DistinctPropertyIterator + propertySet (scheduler/feasible.go:601-704,
scheduler/propertyset.go:14-355).

KATs follow feasible_test.go:1424-2224 (TestDistinctPropertyIterator_*) at the
Stack boundary: state allocs from the store, plan allocs through Commit and
plan stops through StopAllocs (Plan.NodeUpdate). Each runs on the oracle and on
the engine (gpu). The SystemStack has the same iterator (stack.go:252): its
placements are checked against the oracle's node-by-node Selects.
"""
import pytest

from nomad_amd import synth
from nomad_amd.structs import Allocation, Constraint, Job, Task, TaskGroup
from oracle.oracle import OracleGenericStack
from tests.helpers import assert_same_placements, run_place


def _engine(**kw):
    from nomad_amd.stack import GenericStack
    return GenericStack(**kw)


STACKS = [pytest.param(OracleGenericStack, id="oracle"),
          pytest.param(_engine, id="engine", marks=pytest.mark.gpu)]


def rack_nodes(k=5):
    nodes = []
    for i in range(k):
        nd = synth.mock_node("node-%d" % i)
        nd.meta["rack"] = "%d" % i
        nd.compute_class()
        nodes.append(nd)
    return nodes


def two_group_job(job_cons=(), tg_cons=()):
    def tg(name):
        return TaskGroup(name=name, count=1, ephemeral_disk_mb=0, constraints=list(tg_cons),
                         tasks=[Task(name="web", driver="exec", cpu=100, memory_mb=64)])
    return Job(id="foo", constraints=list(job_cons), task_groups=[tg("bar"), tg("baz")])


def alloc(node, job, tg):
    return Allocation(node_id=node, job_id=job, task_group=tg, cpu_shares=100, memory_mb=64)


def feasible_rows(st, nodes, tg):
    """Rows a full pass finds feasible for task group `tg` (one Select per node)."""
    ok = []
    for i, nd in enumerate(nodes):
        st.SetNodes([nd])
        r = st.SelectRaw(tg)
        if r.row >= 0:
            ok.append(i)
    return ok


@pytest.mark.parametrize("stack_cls", STACKS)
def test_job_distinct_property(stack_cls):
    """feasible_test.go:1424-1602: allocs of the job on racks 0-3 (state and
    plan, both task groups) leave only rack 4; other jobs' allocs are ignored."""
    nodes = rack_nodes()
    job = two_group_job(job_cons=[Constraint("${meta.rack}", "", "distinct_property")])
    allocs = [alloc("node-1", "foo", "bar"), alloc("node-1", "ignore 2", "baz"),
              alloc("node-3", "foo", "baz"), alloc("node-3", "ignore 2", "bar")]
    st = stack_cls()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes([nodes[0]])
    st.Commit(0, 0)                 # plan: bar on rack 0
    st.SetNodes([nodes[2]])
    st.Commit(1, 2)                 # plan: baz on rack 2
    assert feasible_rows(st, nodes, 0) == [4]
    assert feasible_rows(st, nodes, 1) == [4]


@pytest.mark.parametrize("stack_cls", STACKS)
def test_job_distinct_property_count(stack_cls):
    """feasible_test.go:1604-1809: RTarget "2" allows two allocs per value."""
    nodes = rack_nodes(3)
    job = two_group_job(job_cons=[Constraint("${meta.rack}", "2", "distinct_property")])
    allocs = [alloc("node-0", "foo", "bar"), alloc("node-0", "foo", "baz"),
              alloc("node-1", "foo", "bar"), alloc("node-2", "other", "bar"),
              alloc("node-2", "other", "bar")]
    st = stack_cls()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    assert feasible_rows(st, nodes, 0) == [1, 2]
    st.SetNodes([nodes[1]])
    st.Commit(1, 1)                 # second alloc on rack 1
    assert feasible_rows(st, nodes, 0) == [2]


@pytest.mark.parametrize("stack_cls", STACKS)
def test_job_distinct_property_infeasible_and_bad_rtarget(stack_cls):
    """feasible_test.go:1893-2063: no value left -> nothing feasible; a node
    without the property is filtered; an RTarget that is not a count filters all."""
    nodes = rack_nodes(2)
    del nodes[1].meta["rack"]
    nodes[1].compute_class()
    job = two_group_job(job_cons=[Constraint("${meta.rack}", "", "distinct_property")])
    st = stack_cls()
    st.SetState(nodes, [alloc("node-0", "foo", "bar")])
    st.SetJob(job)
    assert feasible_rows(st, nodes, 0) == []
    bad = two_group_job(job_cons=[Constraint("${meta.rack}", "two", "distinct_property")])
    st2 = stack_cls()
    st2.SetState(rack_nodes(2), [])
    st2.SetJob(bad)
    assert feasible_rows(st2, rack_nodes(2), 0) == []


@pytest.mark.parametrize("stack_cls", STACKS)
def test_task_group_distinct_property(stack_cls):
    """feasible_test.go:2065-2224: a task-group constraint counts only that
    group's allocs."""
    nodes = rack_nodes(3)
    job = two_group_job(tg_cons=[Constraint("${meta.rack}", "", "distinct_property")])
    allocs = [alloc("node-0", "foo", "bar"), alloc("node-1", "foo", "baz")]
    st = stack_cls()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    assert feasible_rows(st, nodes, 0) == [1, 2]
    assert feasible_rows(st, nodes, 1) == [0, 2]


# ---- GPU parity: count loops with distinct_property ----------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("allowed,count", [("", 120), ("3", 330)])
def test_distinct_property_count_loop(allowed, count):
    nodes, allocs = synth.cluster_c3(3000, seed=12)
    job = synth.job_c2(count)
    job.constraints.append(Constraint("${meta.rack}", allowed, "distinct_property"))
    perm = synth.shuffle(len(nodes), 5)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm)
    _, _, re = run_place(_engine, nodes, allocs, job, perm)
    assert_same_placements(re, ro)


@pytest.mark.gpu
def test_distinct_property_with_spread_full_scan():
    nodes, allocs = synth.cluster_c3(2000, seed=13)
    job = synth.job_c3(150)
    job.task_groups[0].constraints.append(Constraint("${meta.rack}", "2", "distinct_property"))
    perm = synth.shuffle(len(nodes), 6)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm)
    _, _, re = run_place(_engine, nodes, allocs, job, perm)
    assert_same_placements(re, ro)


@pytest.mark.parametrize("stack_cls", STACKS)
def test_job_distinct_property_remove_and_replace(stack_cls):
    # feasible_test.go:1811-1891: the node's only alloc of the job is being
    # stopped while a new one is proposed on it; the cleared value is not
    # discounted (one cleared, one proposed: propertyset.go:199-208), so the
    # rack stays used once and the node is infeasible
    nodes = rack_nodes(1)
    tg = TaskGroup(name="bar", count=2, ephemeral_disk_mb=0,
                   tasks=[Task(name="web", driver="exec", cpu=100, memory_mb=64)])
    job = Job(id="foo", constraints=[Constraint("${meta.rack}", "", "distinct_property")], task_groups=[tg])
    stopping = Allocation(node_id=nodes[0].id, job_id="foo", task_group="bar", cpu_shares=100, memory_mb=64)
    st = stack_cls()
    st.SetState(nodes, [stopping])
    st.SetJob(job)
    st.SetNodes([0])
    st.Commit(0, 0)                 # plan.NodeAllocation: a new alloc of foo/bar on the node
    st.StopAllocs([0])              # plan.NodeUpdate: the state alloc
    assert st.Select(0) is None


@pytest.mark.parametrize("stack_cls", STACKS)
def test_job_distinct_property_stop_frees_the_value(stack_cls):
    # the same node without the proposed alloc: the stop clears the value
    nodes = rack_nodes(1)
    tg = TaskGroup(name="bar", count=1, ephemeral_disk_mb=0,
                   tasks=[Task(name="web", driver="exec", cpu=100, memory_mb=64)])
    job = Job(id="foo", constraints=[Constraint("${meta.rack}", "", "distinct_property")], task_groups=[tg])
    stopping = Allocation(node_id=nodes[0].id, job_id="foo", task_group="bar", cpu_shares=100, memory_mb=64)
    st = stack_cls()
    st.SetState(nodes, [stopping])
    st.SetJob(job)
    st.SetNodes([0])
    assert st.Select(0) is None
    st.StopAllocs([0])
    assert st.Select(0) is not None


def _system_distinct_case(n, seed, allowed, job_level, preempt):
    from nomad_amd.structs import SchedulerConfig
    nodes, allocs = synth.cluster_c4(n, seed=seed)
    for i, nd in enumerate(nodes):
        nd.meta["rack"] = "r%02d" % (i % 37)
        if i % 53 == 0:
            nd.meta.pop("rack")        # missing property: filtered
        nd.compute_class()
    job = synth.mock_system_job()
    c = Constraint("${meta.rack}", str(allowed), "distinct_property")
    if job_level:
        job.constraints.append(c)
    else:
        job.task_groups[0].constraints.append(c)
    # a few of the job's own allocs already use some racks
    for i in range(0, n, 97):
        allocs.append(Allocation(node_id=nodes[i].id, job_id=job.id, task_group=job.task_groups[0].name,
                                 cpu_shares=100, memory_mb=64, disk_mb=10, priority=job.priority))
    return nodes, allocs, job, SchedulerConfig(preempt_system=preempt)


@pytest.mark.parametrize("job_level,preempt", [(False, False), (True, True)])
@pytest.mark.gpu
def test_system_stack_distinct_property(job_level, preempt):
    import numpy as np
    from nomad_amd.stack import SystemStack
    from oracle.oracle import OracleSystemStack
    nodes, allocs, job, cfg = _system_distinct_case(2500, 17, 3, job_level, preempt)
    res = []
    for st in (SystemStack(config=cfg), OracleSystemStack(config=cfg)):
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(np.arange(len(nodes), dtype=np.uint32))
        sc, status, placed = st.SystemPlace(0)
        res.append((np.asarray(status).copy(), np.asarray(sc).copy(), placed))
    (s0, c0, p0), (s1, c1, p1) = res
    assert p0 == p1
    np.testing.assert_array_equal(s0, s1)
    np.testing.assert_array_equal(c0, c1)
    assert (s0 == 1).sum() > len(nodes) // 3      # the racks run out


@pytest.mark.gpu
def test_system_stack_distinct_property_single_selects():
    # SystemScheduler one-node Selects with commits (the pe_select path)
    import numpy as np
    from nomad_amd.stack import SystemStack
    from oracle.oracle import OracleSystemStack
    nodes, allocs, job, cfg = _system_distinct_case(400, 18, 2, False, False)
    out = []
    for st in (SystemStack(config=cfg), OracleSystemStack(config=cfg)):
        st.SetState(nodes, allocs)
        st.SetJob(job)
        seq = []
        for i in range(len(nodes)):
            st.SetNodes(np.asarray([i], dtype=np.uint32))
            r = st.Select(0)
            seq.append(None if r is None else (r.row, r.final_score))
            if r is not None:
                st.Commit(0, r.row)
        out.append(seq)
    assert out[0] == out[1]
