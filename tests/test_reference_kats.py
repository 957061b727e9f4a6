"""Known-answer tests ported from the reference's own test suite.

Each KAT rebuilds the reference test's scenario at the Stack boundary and
asserts the reference's exact expected values. Every test runs against the
oracle (CPU, always) and the HIP engine (marked gpu). Scores are compared with
== exactly like the reference (require.Equal on float64).
"""
import math

import numpy as np
import pytest

from nomad_amd import synth
from nomad_amd.structs import (Affinity, Allocation, Constraint, Job, Node, Spread, SpreadTarget, Task,
                               TaskGroup)
from oracle.oracle import OracleGenericStack


def _engine():
    from nomad_amd.stack import GenericStack
    return GenericStack()


STACKS = [pytest.param(OracleGenericStack, id="oracle"),
          pytest.param(_engine, id="engine", marks=pytest.mark.gpu)]


def mk(stack_cls, nodes, allocs, job):
    st = stack_cls()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    return st


def select_on(st, node, tg=0):
    """Select with SetNodes([node]): the chain's verdict and score parts for one node."""
    st.SetNodes([node])
    return st.SelectRaw(tg)


def plain_node(nid, cpu, mem, rcpu, rmem):
    n = synth.mock_node(nid)
    n.cpu_shares, n.memory_mb, n.reserved_cpu, n.reserved_memory_mb = cpu, mem, rcpu, rmem
    n.disk_mb, n.reserved_disk_mb = 0, 0
    n.compute_class()
    return n


def plain_job(cpu, mem, count=1, disk=0):
    return Job(id="kat", task_groups=[TaskGroup(name="web", count=count, ephemeral_disk_mb=disk,
                                                tasks=[Task(name="web", driver="exec", cpu=cpu, memory_mb=mem)])])


@pytest.mark.parametrize("stack_cls", STACKS)
def test_binpack_no_existing_alloc(stack_cls):
    """rank_test.go:34-137 TestBinPackIterator_NoExistingAlloc: perfect fit scores
    exactly 1.0, the overloaded node is exhausted, the 50% fit is in [0.50, 0.60]."""
    nodes = [plain_node("n0", 2048, 2048, 1024, 1024),   # perfect fit
             plain_node("n1", 1024, 1024, 512, 512),     # overloaded
             plain_node("n2", 4096, 4096, 1024, 1024)]   # 50% fit
    st = mk(stack_cls, nodes, [], plain_job(1024, 1024))
    r0, r1, r2 = (select_on(st, n) for n in nodes)
    assert r0.row == 0 and r0.final_score == 1.0
    assert r1.row == -1 and r1.nodes_exhausted == 1
    assert r2.row == 2 and 0.50 <= r2.final_score <= 0.60


@pytest.mark.parametrize("stack_cls", STACKS)
def test_job_anti_affinity_and_normalization(stack_cls):
    """rank_test.go:1628-1695 (-0.75) and :1744-1807 (-0.875 with the rescheduling penalty)."""
    nodes = [synth.mock_node("n0"), synth.mock_node("n1")]
    allocs = [Allocation(node_id="n0", job_id="foo", task_group="web"),
              Allocation(node_id="n0", job_id="foo", task_group="web"),
              Allocation(node_id="n1", job_id="bar", task_group="web")]
    job = synth.mock_job("foo", count=4)
    st = mk(stack_cls, nodes, allocs, job)
    r0 = select_on(st, nodes[0])
    assert r0.scores[1] == -0.75            # -(collisions+1)/desired_count
    r1 = select_on(st, nodes[1])
    assert len(r1.scores) == 1              # no collision: nothing appended
    # TestScoreNormalizationIterator: anti-affinity -0.75 and penalty -1 average to -0.875
    from nomad_amd.stack import SelectOptions
    st.SetNodes([nodes[0]])
    r = st.Select(0, SelectOptions(penalty_node_ids=["n0"]))
    assert r.scores[1:] == [-0.75, -1.0]
    assert (r.scores[1] + r.scores[2]) / 2 == -0.875
    assert r.final_score == (r.scores[0] + -0.75 + -1.0) / 3


@pytest.mark.parametrize("stack_cls", STACKS)
def test_node_affinity_scores(stack_cls):
    """rank_test.go:1809-1882 TestNodeAffinityIterator: 0.5, -1/3, -1/6, 1/3."""
    nodes = [synth.mock_node("n%d" % i) for i in range(4)]
    nodes[0].attributes["kernel.version"] = "4.9"
    nodes[1].datacenter = "dc2"
    nodes[2].datacenter = "dc2"
    nodes[2].node_class = "large"
    for n in nodes:
        n.compute_class()
    job = synth.mock_job("foo")
    job.task_groups[0].affinities = [
        Affinity("${node.datacenter}", "dc1", "=", 100),
        Affinity("${node.datacenter}", "dc2", "=", -100),
        Affinity("${attr.kernel.version}", ">4.0", "version", 50),
        Affinity("${node.class}", "large", "is", 50),
    ]
    job.task_groups[0].network = None
    st = mk(stack_cls, nodes, [], job)
    expected = [0.5, -(1.0 / 3.0), -(1.0 / 6.0), 1.0 / 3.0]
    for n, want in zip(nodes, expected):
        r = select_on(st, n)
        assert r.scores[-1] == want, (n.id, r.scores)


@pytest.mark.parametrize("stack_cls", STACKS)
def test_spread_single_attribute(stack_cls):
    """spread_test.go:15-171 TestSpreadIterator_SingleAttribute: 0.625 / 0.5, then 0 / 0.5."""
    dcs = ["dc1", "dc2", "dc1", "dc1"]
    nodes = []
    for i, dc in enumerate(dcs):
        n = synth.mock_node("n%d" % i)
        n.datacenter = dc
        n.compute_class()
        nodes.append(n)
    job = synth.mock_job("spreadjob", count=10)
    job.task_groups[0].network = None
    job.task_groups[0].spreads = [Spread("${node.datacenter}", 100, [SpreadTarget("dc1", 80)])]
    allocs = [Allocation(node_id="n0", job_id=job.id, task_group="web"),
              Allocation(node_id="n2", job_id=job.id, task_group="web")]
    st = mk(stack_cls, nodes, allocs, job)
    want = {"dc1": 0.625, "dc2": 0.5}
    for n in nodes:
        r = select_on(st, n)
        assert r.scores[-1] == want[n.datacenter], (n.id, r.scores)
    # plan: two more on n0, three on n3 -> dc1 reaches its desired count
    for row in (0, 0, 3, 3, 3):
        st.Commit(0, row)
    for n in nodes:
        r = select_on(st, n)
        if n.datacenter == "dc1":
            assert len(r.scores) == 2 and r.scores[1] < 0   # anti-affinity only, spread 0 not appended
        else:
            assert r.scores[-1] == 0.5


@pytest.mark.parametrize("stack_cls", STACKS)
def test_stack_limit_and_constraint_filter(stack_cls):
    """stack_test.go:57-82 (limit 3 for 8 nodes) and :310-348 (constraint filter metrics)."""
    nodes = [synth.mock_node("n%d" % i) for i in range(8)]
    st = mk(stack_cls, nodes, [], synth.mock_job())
    assert st.SetNodes(nodes) == 3
    nodes2 = [synth.mock_node("a"), synth.mock_node("b")]
    nodes2[0].attributes["kernel.name"] = "freebsd"
    nodes2[0].compute_class()
    job = synth.mock_job()
    job.constraints[0].rtarget = "freebsd"
    st2 = mk(stack_cls, nodes2, [], job)
    st2.SetNodes(nodes2)
    r = st2.SelectRaw(0)
    assert r.row == 0
    assert r.nodes_filtered == 1


@pytest.mark.parametrize("stack_cls", STACKS)
def test_drivers_and_distinct_hosts(stack_cls):
    """DriverChecker (feasible_test.go:767-900) and distinct_hosts (feasible_test.go:1231-1390)."""
    nodes = [synth.mock_node("n%d" % i) for i in range(3)]
    nodes[1].drivers = {}
    nodes[1].attributes.pop("driver.exec")
    nodes[1].compute_class()
    nodes[2].attributes["kernel.name"] = "linux"
    job = synth.mock_job("dh", count=3)
    job.task_groups[0].network = None
    job.constraints.append(Constraint("", "", "distinct_hosts"))
    allocs = [Allocation(node_id="n2", job_id="dh", task_group="other")]
    st = mk(stack_cls, nodes, allocs, job)
    st.SetNodes(nodes)
    r = st.SelectRaw(0)
    assert r.row == 0            # n1 lacks the exec driver, n2 already runs an alloc of the job
    st.Commit(0, 0)
    st.SetNodes(nodes)
    r = st.SelectRaw(0)
    assert r.row == -1 and r.nodes_filtered == 3


def _core_node(nid, reservable=(0, 1)):
    n = plain_node(nid, 2048, 2048, 0, 0)
    n.total_cores = 2
    n.reservable_cores = list(reservable)
    n.compute_class()
    return n


@pytest.mark.parametrize("stack_cls", STACKS)
def test_binpack_reserved_cores(stack_cls):
    """rank_test.go:950-1065 TestBinPackIterator_ReservedCores: the node whose
    cores are both held is exhausted ("cores"); the other one is picked and the
    task gets core 1."""
    nodes = [_core_node("n0"), _core_node("n1")]
    allocs = [Allocation(node_id="n0", job_id="j1", task_group="web", cpu_shares=2048, memory_mb=2048,
                         reserved_cores=[0, 1]),
              Allocation(node_id="n1", job_id="j2", task_group="web", cpu_shares=1024, memory_mb=1024,
                         reserved_cores=[0])]
    job = Job(id="kat", task_groups=[TaskGroup(name="web", count=1, ephemeral_disk_mb=0, tasks=[
        Task(name="web", driver="exec", cpu=0, memory_mb=1024, cores=1)])])
    st = mk(stack_cls, nodes, allocs, job)
    st.SetNodes(nodes)
    r = st.SelectRaw(0)
    assert r.row == 1 and r.reserved_cores == [1]
    assert r.nodes_exhausted == 1
    st.SetNodes([nodes[0]])
    assert st.SelectRaw(0).row == -1
