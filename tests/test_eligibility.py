"""EvalEligibility export (pe_get_eligibility) against the oracle's memo.

After an evaluation's Selects the reference's ctx.Eligibility() holds the
job-level and per task group ComputedClassFeasibility entries that
FeasibilityWrapper.Next wrote for every node the chain pulled
(scheduler/feasible.go:1061-1153, context.go:190-356). GenericScheduler hands
GetClasses() and HasEscaped() to blocked evaluations
(generic_sched.go:177-181, 193-203). The engine emulates the memo internally;
these tests check that what it exports equals the oracle chain's memo, entry
for entry, over windowed, full-pass, preferred-node, escaped, multi task group,
preemption and SystemStack evaluations (VERDICT r02 boundary gap 1).
"""
import dataclasses

import numpy as np
import pytest

from nomad_amd import synth
from nomad_amd.stack import SelectOptions
from nomad_amd.structs import Constraint, DriverInfo, SchedulerConfig, Spread, SpreadTarget, Task, TaskGroup
from oracle.oracle import OracleGenericStack, OracleSystemStack
from tests.helpers import assert_same_placements

pytestmark = pytest.mark.gpu


def engine_generic(**kw):
    from nomad_amd.stack import GenericStack
    return GenericStack(**kw)


def engine_system(**kw):
    from nomad_amd.stack import SystemStack
    return SystemStack(**kw)


def mixed_cluster(n, seed=42):
    """C2 nodes with classes that fail the job constraint (windows) and nodes
    that fail a task-group check (no exec driver; drivers are not hashed into
    the class, so some classes are non-uniform)."""
    nodes, allocs = synth.cluster_c2(n, seed=seed)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    for nd in nodes:
        u = rng.random()
        if u < 0.2:
            nd.attributes["kernel.name"] = "windows"
        if rng.random() < 0.15:
            nd.drivers = {k: v for k, v in nd.drivers.items() if k != "exec"}
            nd.drivers["docker"] = DriverInfo()
            nd.attributes.pop("driver.exec", None)
        if rng.random() < 0.1:
            nd.node_class = "special"
        nd.compute_class()
    return nodes, allocs


def pair(stack_e, stack_o, nodes, allocs, job, perm):
    for st in (stack_e, stack_o):
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(list(perm))


def assert_same_eligibility(e, o):
    ee, oe = e.Eligibility(), o.Eligibility()
    assert ee["job"] == oe["job"]
    assert ee["tgs"] == oe["tgs"]
    assert ee["escaped"] == oe["escaped"]
    assert e.GetClasses(ee) == o.GetClasses(oe)
    return ee


def select_commit(e, o, tg, k, opts=None):
    for _ in range(k):
        a, b = o.SelectRaw(tg, opts), e.SelectRaw(tg, opts)
        assert_same_placements([b], [a])
        if a.row < 0:
            return False
        o.Commit(tg, a.row)
        e.Commit(tg, b.row)
    return True


def test_windowed_select_commit_and_place():
    nodes, allocs = mixed_cluster(2000)
    job = synth.job_c2(300)
    perm = synth.shuffle(len(nodes), 3)
    e, o = engine_generic(), OracleGenericStack()
    pair(e, o, nodes, allocs, job, perm)
    assert_same_eligibility(e, o)          # nothing visited yet: empty maps
    select_commit(e, o, 0, 1)
    ee = assert_same_eligibility(e, o)
    assert ee["job"] and ee["tgs"]["web"]
    select_commit(e, o, 0, 40)              # served from the speculative count loop
    assert_same_eligibility(e, o)
    ro, re_ = o.Place(0, 200), e.Place(0, 200)
    assert_same_placements(re_, ro)
    ee = assert_same_eligibility(e, o)
    assert False in ee["tgs"]["web"].values() and False in ee["job"].values()


def test_blocked_eval_nothing_fits():
    """A job no node can hold: the nil Select pulls the whole list, so every
    class ends in the maps (what the blocked eval's ClassEligibility gets)."""
    nodes, allocs = mixed_cluster(1500, seed=5)
    job = synth.job_c2(10)
    job.task_groups[0].tasks[0].cpu = 10 ** 6
    perm = synth.shuffle(len(nodes), 4)
    e, o = engine_generic(), OracleGenericStack()
    pair(e, o, nodes, allocs, job, perm)
    assert not select_commit(e, o, 0, 1)
    ee = assert_same_eligibility(e, o)
    classes = {nd.computed_class for nd in nodes}
    assert set(ee["job"]) == classes


def test_full_pass_and_escaped_job():
    nodes, allocs = synth.cluster_c3(3000, seed=7)
    job = synth.job_c3(50)
    job = dataclasses.replace(job, constraints=job.constraints + [
        Constraint("${node.unique.name}", "node-00007", "!=")])
    perm = synth.shuffle(len(nodes), 2)
    e, o = engine_generic(), OracleGenericStack()
    pair(e, o, nodes, allocs, job, perm)
    select_commit(e, o, 0, 20)
    ee = assert_same_eligibility(e, o)
    assert ee["escaped"] and not ee["job"] and ee["tgs"]["web"]


def test_preferred_nodes_and_penalties():
    nodes, allocs = mixed_cluster(1200, seed=9)
    job = synth.job_c2(50)
    perm = synth.shuffle(len(nodes), 6)
    e, o = engine_generic(), OracleGenericStack()
    pair(e, o, nodes, allocs, job, perm)
    pref = SelectOptions(preferred_nodes=[nodes[17].id, nodes[900].id, nodes[31].id])
    a, b = o.Select(0, pref), e.Select(0, pref)
    assert (a.row if a else -1) == (b.row if b else -1)
    assert_same_eligibility(e, o)
    if a:
        o.Commit(0, a.row)
        e.Commit(0, b.row)
    select_commit(e, o, 0, 10)
    assert_same_eligibility(e, o)


def test_two_task_groups_with_spreads_interleaved():
    """Two groups with spreads: SpreadIterator.sumSpreadWeights accumulates
    over groups (spread.go:254) and Next divides by the running sum
    (spread.go:157), so group A's scores change once group B has selected."""
    nodes, allocs = synth.cluster_c3(2000, seed=11)
    base = synth.job_c3(30)
    tg_a = base.task_groups[0]
    tg_b = TaskGroup(name="api", count=30, ephemeral_disk_mb=150,
                     constraints=[Constraint("${attr.kernel.name}", "linux", "=")],
                     spreads=[Spread("${meta.rack}", 40, [SpreadTarget("r01", 50)])],
                     tasks=[Task(name="api", driver="exec", cpu=300, memory_mb=200)])
    tg_a = dataclasses.replace(tg_a, spreads=[Spread("${node.class}", 70, [])])
    job = dataclasses.replace(base, task_groups=[tg_a, tg_b])
    perm = synth.shuffle(len(nodes), 12)
    e, o = engine_generic(), OracleGenericStack()
    pair(e, o, nodes, allocs, job, perm)
    for _ in range(12):
        select_commit(e, o, 0, 1)
        select_commit(e, o, 1, 1)
    assert_same_eligibility(e, o)


def test_preemption_count_loop():
    nodes, allocs = synth.cluster_c5(3000, seed=3, busy=0.99)
    job = synth.job_c5(200)
    perm = synth.shuffle(len(nodes), 5)
    cfg = SchedulerConfig(preempt_service=True)
    e, o = engine_generic(config=cfg), OracleGenericStack(config=cfg)
    pair(e, o, nodes, allocs, job, perm)
    ro, re_ = o.Place(0, 200), e.Place(0, 200)
    assert_same_placements(re_, ro)
    assert_same_eligibility(e, o)


def test_system_stack_single_node_selects():
    """SystemScheduler.computePlacements: SetNodes([node]) + Select per node
    (scheduler_system.go:289-302)."""
    nodes, allocs = mixed_cluster(400, seed=13)
    job = synth.mock_system_job()
    e, o = engine_system(), OracleSystemStack()
    for st in (e, o):
        st.SetState(nodes, allocs)
        st.SetJob(job)
    for k in range(0, 400, 3):
        for st in (e, o):
            st.SetNodes([k])
        a, b = o.SelectRaw(0), e.SelectRaw(0)
        assert a.row == b.row
        if a.row >= 0:
            o.Commit(0, a.row)
            e.Commit(0, b.row)
    assert_same_eligibility(e, o)


def test_changed_only_deltas_rebuild_the_maps():
    """The shim's per-Select mirror: applying the changed entries after every
    Select rebuilds exactly the full maps."""
    nodes, allocs = mixed_cluster(1500, seed=21)
    job = synth.job_c2(100)
    perm = synth.shuffle(len(nodes), 8)
    e, o = engine_generic(), OracleGenericStack()
    pair(e, o, nodes, allocs, job, perm)
    mirror = {"job": {}, "tgs": {}}
    for _ in range(60):
        if not select_commit(e, o, 0, 1):
            break
        d = e.Eligibility(changed_only=True)
        mirror["job"].update(d["job"])
        for tg, m in d["tgs"].items():
            mirror["tgs"].setdefault(tg, {}).update(m)
    full = e.Eligibility()
    assert mirror["job"] == full["job"] and mirror["tgs"] == full["tgs"]
    assert_same_eligibility(e, o)
