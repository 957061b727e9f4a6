"""Incremental snapshot updates (SoA ingest): an
allocation delta of the state store (allocs turning terminal — client status
complete / failed / lost — and allocs placed by other workers' applied plans,
nomad/state UpsertAllocs / UpsertPlanResults) applied to the resident HBM
snapshot with pe_update_allocs must behave exactly like a full pe_set_state of
the updated tables: same placements, scores, metrics counters, preemptions.
The reference is the oracle run on the updated state from scratch.
"""
import copy
import random

import pytest

from nomad_amd import synth
from nomad_amd.structs import Allocation, SchedulerConfig
from oracle.oracle import OracleGenericStack
from tests.helpers import assert_same_placements, run_place


def _delta(nodes, allocs, seed, frac_terminal=0.3, n_new=150):
    rng = random.Random(seed)
    changed, index = [], []
    for i, a in enumerate(allocs):
        if not a.terminal and rng.random() < frac_terminal:
            b = copy.deepcopy(a)
            b.terminal = True
            changed.append(b)
            index.append(i)
    for k in range(n_new):
        nd = rng.choice(nodes)
        changed.append(Allocation(node_id=nd.id, job_id="other-%d" % (k % 7), task_group="web",
                                  cpu_shares=rng.choice([250, 500, 1000]), memory_mb=rng.choice([128, 512]),
                                  disk_mb=150, priority=rng.choice([20, 50])))
        index.append(None)
    updated = list(allocs)
    for a, i in zip(changed, index):
        if i is None:
            updated.append(a)
        else:
            updated[i] = a
    return changed, index, updated


@pytest.mark.gpu
def test_update_allocs_equals_fresh_state():
    from nomad_amd.stack import GenericStack
    nodes, allocs = synth.cluster_c2(1500, seed=21)
    changed, index, updated = _delta(nodes, allocs, 1)
    job = synth.job_c2(300)
    perm = synth.shuffle(len(nodes), 7)
    st = GenericStack()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes(list(perm))
    st.Place(0, 50)                      # an evaluation on the old snapshot
    st.UpdateAllocs(changed, index)      # state delta: plan / memo / job reset
    st.SetJob(job)
    st.SetNodes(list(perm))
    got = st.Place(0, 300)
    _, _, want = run_place(OracleGenericStack, nodes, updated, job, perm)
    assert_same_placements(got, want)
    # a second delta on top of the first
    changed2, index2, updated2 = _delta(nodes, updated, 2, frac_terminal=0.2, n_new=80)
    st.UpdateAllocs(changed2, index2)
    st.SetJob(job)
    st.SetNodes(list(perm))
    got2 = st.Place(0, 300)
    _, _, want2 = run_place(OracleGenericStack, nodes, updated2, job, perm)
    assert_same_placements(got2, want2)


@pytest.mark.gpu
def test_update_allocs_devices_and_preemption():
    # device holders turning terminal free instances; new low-priority holders
    # become preemption candidates (PreemptForDevice / PreemptForTaskGroup)
    from nomad_amd.stack import GenericStack
    cfg = SchedulerConfig(preempt_service=True)
    nodes, allocs = synth.cluster_c5(600, seed=4, busy=0.9)
    rng = random.Random(5)
    changed, index = [], []
    for i, a in enumerate(allocs):
        if a.devices and not a.terminal and rng.random() < 0.25:
            b = copy.deepcopy(a)
            b.terminal = True
            changed.append(b)
            index.append(i)
    updated = list(allocs)
    for a, i in zip(changed, index):
        updated[i] = a
    job = synth.job_c5(120)
    perm = synth.shuffle(len(nodes), 9)
    st = GenericStack(config=cfg)
    st.SetState(nodes, allocs)
    st.UpdateAllocs(changed, index)
    st.SetJob(job)
    st.SetNodes(list(perm))
    got = st.Place(0, 120)
    _, _, want = run_place(OracleGenericStack, nodes, updated, job, perm, config=cfg)
    assert_same_placements(got, want)
    assert [g.preempted for g in got] == [w.preempted for w in want]


def _node_delta(nodes, seed, n_changed=120, n_new=40, devices=False):
    """Node upserts: capacity, attribute (class), driver and device changes on
    existing rows, plus new nodes appended."""
    rng = random.Random(seed)
    changed, index = [], []
    for r in rng.sample(range(len(nodes)), n_changed):
        nd = copy.deepcopy(nodes[r])
        k = rng.randrange(4)
        if k == 0:
            nd.cpu_shares = rng.choice([8000, 16000])
        elif k == 1:
            nd.attributes["kernel.name"] = rng.choice(["linux", "windows"])
            nd.node_class = "class-%d" % rng.randrange(12)
        elif k == 2:
            nd.drivers = {}
            nd.attributes.pop("driver.exec", None)
        elif devices and nd.devices:
            nd.devices[0].healthy = max(0, nd.devices[0].healthy - 2)
        else:
            nd.meta["rack"] = "r%d" % rng.randrange(5)
        nd.compute_class()
        changed.append(nd)
        index.append(r)
    base = synth.cluster_c5(n_new, seed=seed + 100)[0] if devices else synth.cluster_c2(n_new, seed=seed + 100)[0]
    for nd in base:
        nd.id = "new-" + nd.id
        nd.compute_class()
        changed.append(nd)
        index.append(None)
    updated = list(nodes)
    for nd, r in zip(changed, index):
        if r is None:
            updated.append(nd)
        else:
            updated[r] = nd
    return changed, index, updated


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["c2", "c3"])
def test_update_nodes_equals_fresh_state(kind):
    from nomad_amd.stack import GenericStack
    if kind == "c2":
        nodes, allocs = synth.cluster_c2(1500, seed=31)
        job = synth.job_c2(300)
    else:
        nodes, allocs = synth.cluster_c3(1500, seed=32)
        job = synth.job_c3(200)
    changed, index, updated = _node_delta(nodes, 3)
    st = GenericStack()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes(synth.shuffle(len(nodes), 5))
    st.Place(0, 40)                       # an evaluation on the old snapshot
    st.UpdateNodes(changed, index)        # node upserts: rows replaced and appended
    perm = synth.shuffle(len(updated), 6)
    st.SetJob(job)
    st.SetNodes(list(perm))
    got = st.Place(0, job.task_groups[0].count)
    _, _, want = run_place(OracleGenericStack, updated, allocs, job, perm)
    assert_same_placements(got, want)
    # then an alloc delta on the updated snapshot, and a second node delta
    changed2, index2, updated2 = _delta(updated, allocs, 4, frac_terminal=0.2, n_new=60)
    st.UpdateAllocs(changed2, index2)
    changed3, index3, updated3 = _node_delta(updated, 7, n_changed=60, n_new=10)
    st.UpdateNodes(changed3, index3)
    perm3 = synth.shuffle(len(updated3), 8)
    st.SetJob(job)
    st.SetNodes(list(perm3))
    got3 = st.Place(0, job.task_groups[0].count)
    _, _, want3 = run_place(OracleGenericStack, updated3, updated2, job, perm3)
    assert_same_placements(got3, want3)


@pytest.mark.gpu
def test_update_nodes_devices_and_preemption():
    from nomad_amd.stack import GenericStack
    cfg = SchedulerConfig(preempt_service=True)
    nodes, allocs = synth.cluster_c5(700, seed=33, busy=0.8)
    changed, index, updated = _node_delta(nodes, 9, n_changed=150, n_new=30, devices=True)
    job = synth.job_c5(100)
    perm = synth.shuffle(len(updated), 10)
    st = GenericStack(config=cfg)
    st.SetState(nodes, allocs)
    st.UpdateNodes(changed, index)
    st.SetJob(job)
    st.SetNodes(list(perm))
    got = st.Place(0, 100)
    _, _, want = run_place(OracleGenericStack, updated, allocs, job, perm, config=cfg)
    assert_same_placements(got, want)
    assert [g.preempted for g in got] == [w.preempted for w in want]


@pytest.mark.gpu
def test_update_nodes_many_rounds_lists_move_and_compact():
    """pe_update_nodes rewrites a changed row's lists in place when they do not
    grow and moves them to the end of their vector when they do; dead ranges
    are compacted once they outnumber the live ones. Six rounds of upserts
    that add attributes / meta / drivers (lists grow), drop them (lists
    shrink), flip classes and append nodes, on one handle; every round equals
    the oracle on the updated snapshot from scratch."""
    from nomad_amd.stack import GenericStack
    nodes, allocs = synth.cluster_c3(1200, seed=41)
    job = synth.job_c3(60)
    st = GenericStack()
    st.SetState(nodes, allocs)
    cur = list(nodes)
    rng = random.Random(17)
    for rnd in range(6):
        changed, index = [], []
        for r in rng.sample(range(len(cur)), 400):
            nd = copy.deepcopy(cur[r])
            k = (r + rnd) % 4
            if k == 0:   # longer attribute and meta lists
                for q in range(rnd + 2):
                    nd.attributes["extra.%d.%d" % (rnd, q)] = "v%d" % q
                nd.meta["zone%d" % rnd] = "z%d" % (r % 3)
            elif k == 1:   # shorter lists
                for key in [a for a in nd.attributes if a.startswith("extra.")][:3]:
                    nd.attributes.pop(key)
                nd.meta.pop("rack", None)
            elif k == 2:
                nd.attributes["kernel.name"] = rng.choice(["linux", "windows"])
                nd.drivers = dict(nd.drivers)
            else:
                nd.cpu_shares = rng.choice([4000, 8000, 16000])
            nd.compute_class()
            changed.append(nd)
            index.append(r)
        for q in range(25):
            nd = copy.deepcopy(cur[rng.randrange(len(cur))])
            nd.id = "joined-%d-%d" % (rnd, q)
            nd.compute_class()
            changed.append(nd)
            index.append(None)
        for nd, r in zip(changed, index):
            if r is None:
                cur.append(nd)
            else:
                cur[r] = nd
        st.UpdateNodes(changed, index)
        perm = synth.shuffle(len(cur), 50 + rnd)
        st.SetJob(job)
        st.SetNodes(list(perm))
        got = st.Place(0, 60)
        _, _, want = run_place(OracleGenericStack, cur, allocs, job, perm)
        assert_same_placements(got, want)


@pytest.mark.gpu
def test_checker_caches_across_jobs():
    """The engine reuses per-class checker results of earlier SetJobs on the
    same node table (job constraints, task-group checkers, node affinities,
    spread values). Jobs that differ in one constraint, in an
    affinity weight or in the spread target, set in turn on one stack, each
    place exactly as a fresh oracle does; a node update in between drops the
    caches."""
    from nomad_amd.stack import GenericStack
    from nomad_amd.structs import Affinity, Constraint, Spread, SpreadTarget
    nodes, allocs = synth.cluster_c3(1500, seed=41)
    a = synth.job_c3(60)
    b = copy.deepcopy(a)
    b.id = "svc-b"
    b.constraints[2] = Constraint("${meta.rack}", "^r[5-9]", "regexp")
    c = copy.deepcopy(a)
    c.id = "svc-c"
    c.affinities = [Affinity("${node.class}", "c3", "=", 80)]
    d = copy.deepcopy(a)
    d.id = "svc-d"
    d.spreads = [Spread("${attr.os.version}", 100, [SpreadTarget("5.4.0", 40), SpreadTarget("5.10.12", 40)])]
    st = GenericStack()
    st.SetState(nodes, allocs)
    state = nodes
    for k, job in enumerate([a, b, a, c, d, a, "update", b, a]):
        if job == "update":
            changed, index, state = _node_delta(state, 9, n_changed=80, n_new=5)
            st.UpdateNodes(changed, index)
            continue
        st.ResetPlan()
        st.SetJob(job)
        perm = synth.shuffle(len(state), 20 + k)
        st.SetNodes(list(perm))
        got = st.Place(0, job.task_groups[0].count)
        _, _, want = run_place(OracleGenericStack, state, allocs, job, perm)
        assert_same_placements(got, want)


@pytest.mark.gpu
def test_job_checker_rows_across_jobs_metrics():
    """The per-row job checker outcomes (the FilterNode reasons of
    FeasibilityWrapper's job checkers, feasible.go:1086-1097) are kept across
    evaluations of jobs with the same constraints and dropped when a
    constraint text or the node table changes: every Select's AllocMetric maps
    equal a fresh oracle's, jobs set in turn on one stack."""
    from nomad_amd.stack import GenericStack
    from nomad_amd.structs import Constraint
    nodes, allocs = synth.cluster_c3(1200, seed=43)
    a = synth.job_c3(40)
    b = copy.deepcopy(a)
    b.id = "svc-b"
    b.constraints[2] = Constraint("${meta.rack}", "^r[5-9]", "regexp")
    st = GenericStack()
    st.SetState(nodes, allocs)
    st.EnableMetrics(True)
    state = nodes
    for k, job in enumerate([a, a, b, a, "update", a, b]):
        if job == "update":
            changed, index, state = _node_delta(state, 5, n_changed=120, n_new=4)
            st.UpdateNodes(changed, index)
            continue
        st.ResetPlan()
        st.SetJob(job)
        perm = list(synth.shuffle(len(state), 60 + k))
        st.SetNodes(perm)
        o = OracleGenericStack()
        o.SetState(state, allocs)
        o.SetJob(job)
        o.SetNodes(perm)
        o.EnableMetrics(True)
        for _ in range(25):
            ro, re = o.SelectRaw(0), st.SelectRaw(0)
            assert_same_placements([re], [ro])
            assert st.LastMetrics() == o.LastMetrics()
            if ro.row < 0:
                break
            o.Commit(0, ro.row)
            st.Commit(0, ro.row)
