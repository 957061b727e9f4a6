"""The unchanged caller through the shim (nomad_amd/shim.py, the Python mirror
of INTEGRATION.md's Go shim): computePlacements (generic_sched.go:472-652)
below only calls SetNodes / Select and mutates the plan (AppendStoppedAlloc
for destructive updates, PopUpdate when the replacement fails,
AppendPreemptedAlloc + AppendAlloc); the shim replays the plan into the engine
before each stack call. The engine behind the shim must equal the oracle
behind the shim and the oracle driven call by call (the plan mutations applied
the moment the caller makes them), Select by Select, across evaluations on one
resident handle."""
import numpy as np
import pytest

from nomad_amd import synth
from nomad_amd.shim import DeviceStack, Plan, PlanAlloc
from nomad_amd.stack import SelectOptions
from nomad_amd.structs import Allocation, SchedulerConfig
from oracle.oracle import OracleGenericStack


def _key(r):
    if r is None:
        return None
    return (r.row, r.final_score, tuple(r.scores), r.nodes_evaluated, r.nodes_exhausted, r.new_offset,
            tuple(r.preempted))


class _Direct:
    """The oracle with every plan mutation applied as the caller makes it."""

    def __init__(self, st):
        self.st = st

    def stop(self, a):
        self.st.StopAllocs([a])

    def pop(self, a):
        self.st.PopUpdate(a)

    def place(self, tg, option):
        self.st.Commit(tg, option.row, option.preempted)


def compute_placements(stack, plan, job, place, rows, row_of_alloc, preempt, direct=None, eval_no=0):
    """generic_sched.go:472-652 restated: `place` lists (task group, previous
    alloc row or None); the caller never talks to the engine directly."""
    stack.SetNodes(rows)
    failed = set()
    out = []
    for i, (tg, prev) in enumerate(place):
        if tg in failed:                     # failedTGAllocs short-circuit (:519-523)
            continue
        if prev is not None:                 # stop the previous allocation (:541-547)
            plan.AppendStoppedAlloc(prev, row_of_alloc[prev])
            if direct:
                direct.stop(prev)
        option = stack.Select(tg)            # selectNextOption (:773-792)
        if option is None and preempt:
            option = stack.Select(tg, SelectOptions(preempt=True))
        out.append(_key(option))
        if option is None:
            failed.add(tg)
            if prev is not None:             # undo the stop (:642-645)
                plan.PopUpdate(prev, row_of_alloc[prev])
                if direct:
                    direct.pop(prev)
            continue
        alloc = PlanAlloc(id="e%d-a%d" % (eval_no, i), node_row=option.row, task_group=tg)
        for p in option.preempted:           # handlePreemptions (:794-816)
            plan.AppendPreemptedAlloc(p, row_of_alloc[p], alloc.id)
        plan.AppendAlloc(alloc)              # (:627)
        if direct:
            direct.place(tg, option)
    return out


def _cluster(n, seed, own, busy=0.0, c5=False):
    if c5:
        nodes, allocs = synth.cluster_c5(n, seed=seed, busy=busy)
        job = synth.job_c5(own)
        tg = "infer"
    else:
        nodes, allocs = synth.cluster_c2(n, seed=seed)
        job = synth.job_c2(own)
        tg = "web"
    rng = np.random.Generator(np.random.PCG64(seed))
    for k in rng.choice(n, size=own, replace=False):
        allocs.append(Allocation(node_id=nodes[int(k)].id, job_id=job.id, task_group=tg, cpu_shares=400,
                                 memory_mb=256, disk_mb=150, priority=job.priority))
    return nodes, allocs, job, tg


def _run(make_stack, nodes, allocs, job, tg, evals, config=None):
    st = make_stack(config)
    st.SetState(nodes, allocs)
    row_of = {i: st.row(a.node_id) for i, a in enumerate(allocs)}
    own = [i for i, a in enumerate(allocs) if a.job_id == job.id]
    shim = DeviceStack(st, Plan())
    seqs = []
    for e, (seed, n_new, n_destr) in enumerate(evals):
        plan = Plan()
        if e:
            shim.new_eval(plan)
        else:
            shim.plan = plan
        shim.SetJob(job)
        place = [(tg, own[(e * 7 + k) % len(own)]) for k in range(n_destr)] + [(tg, None)] * n_new
        seqs.append(compute_placements(shim, plan, job, place, synth.shuffle(len(nodes), seed), row_of,
                                       config is not None, eval_no=e))
    return seqs


def _oracle(config):
    return OracleGenericStack(config=config)


def _engine(config):
    from nomad_amd.stack import GenericStack
    return GenericStack(config=config)


EVALS = [(101, 150, 40), (102, 80, 120), (103, 300, 0)]


def _direct_oracle(nodes, allocs, job, tg, evals, config=None):
    """Oracle driven call by call, plan mutations applied immediately (no shim replay)."""
    st = _oracle(config)
    st.SetState(nodes, allocs)
    row_of = {i: st.row(a.node_id) for i, a in enumerate(allocs)}
    own = [i for i, a in enumerate(allocs) if a.job_id == job.id]
    seqs = []

    class _Raw:
        def SetNodes(self, rows):
            return st.SetNodes(rows)

        def Select(self, tg_, options=None):
            return st.Select(tg_, options)
    for e, (seed, n_new, n_destr) in enumerate(evals):
        if e:
            st.ResetPlan()
        st.SetJob(job)
        place = [(tg, own[(e * 7 + k) % len(own)]) for k in range(n_destr)] + [(tg, None)] * n_new
        seqs.append(compute_placements(_Raw(), Plan(), job, place, synth.shuffle(len(nodes), seed), row_of,
                                       config is not None, direct=_Direct(st), eval_no=e))
    return seqs


def test_shim_replay_equals_direct_calls_on_oracle():
    nodes, allocs, job, tg = _cluster(1200, 71, 200)
    assert _run(_oracle, nodes, allocs, job, tg, EVALS) == _direct_oracle(nodes, allocs, job, tg, EVALS)


def test_shim_replay_with_preemption_on_oracle():
    nodes, allocs, job, tg = _cluster(500, 72, 60, busy=0.9, c5=True)
    cfg = SchedulerConfig(preempt_service=True)
    ev = [(201, 70, 20), (202, 40, 10)]
    assert _run(_oracle, nodes, allocs, job, tg, ev, cfg) == _direct_oracle(nodes, allocs, job, tg, ev, cfg)


@pytest.mark.gpu
def test_engine_behind_the_shim():
    nodes, allocs, job, tg = _cluster(3000, 73, 400)
    assert _run(_engine, nodes, allocs, job, tg, EVALS) == _direct_oracle(nodes, allocs, job, tg, EVALS)


@pytest.mark.gpu
def test_engine_behind_the_shim_with_preemption():
    nodes, allocs, job, tg = _cluster(900, 74, 80, busy=0.9, c5=True)
    cfg = SchedulerConfig(preempt_service=True)
    ev = [(301, 90, 30), (302, 60, 20)]
    assert _run(_engine, nodes, allocs, job, tg, ev, cfg) == _direct_oracle(nodes, allocs, job, tg, ev, cfg)


# ---- fallback hand-off (PE_EUNSUPPORTED mid-evaluation) ---------------------

class _FlakyOracle:
    """The oracle as the product side, answering every k-th Select with
    Unsupported (CPU stand-in for the engine's PE_TEST_FALLBACK_EVERY hook)."""

    def __init__(self, config, every):
        self.st = OracleGenericStack(config=config)
        self.every, self.calls = every, 0

    def __getattr__(self, name):
        return getattr(self.st, name)

    def Select(self, tg, options=None):
        from nomad_amd.stack import Unsupported
        self.calls += 1
        if self.calls % self.every == 0:
            raise Unsupported(-4, "test")
        return self.st.Select(tg, options)


def _run_fb(make_stack, nodes, allocs, job, evals, tgs, config=None):
    """Like _run, with a fallback reference chain behind the shim; `tgs` cycles
    the task groups of the fresh placements (interleaved groups)."""
    st = make_stack(config)
    st.SetState(nodes, allocs)
    fb = OracleGenericStack(config=config)
    fb.SetState(nodes, allocs)
    row_of = {i: st.row(a.node_id) for i, a in enumerate(allocs)}
    own = [i for i, a in enumerate(allocs) if a.job_id == job.id]
    shim = DeviceStack(st, Plan(), fallback=fb)
    seqs, eligs = [], []
    for e, (seed, n_new, n_destr) in enumerate(evals):
        plan = Plan()
        if e:
            shim.new_eval(plan)
        else:
            shim.plan = plan
        shim.SetJob(job)
        place = [(tgs[0], own[(e * 7 + k) % len(own)]) for k in range(n_destr)] + \
                [(tgs[k % len(tgs)], None) for k in range(n_new)]
        seqs.append(compute_placements(shim, plan, job, place, synth.shuffle(len(nodes), seed), row_of,
                                       config is not None, eval_no=e))
        eligs.append(shim.ctx_eligibility)
    return seqs, eligs, shim.fallback_selects


def _direct_fb(nodes, allocs, job, evals, tgs, config=None):
    st = _oracle(config)
    st.SetState(nodes, allocs)
    row_of = {i: st.row(a.node_id) for i, a in enumerate(allocs)}
    own = [i for i, a in enumerate(allocs) if a.job_id == job.id]
    seqs, eligs = [], []

    class _Raw:
        def SetNodes(self, rows):
            return st.SetNodes(rows)

        def Select(self, tg_, options=None):
            return st.Select(tg_, options)
    for e, (seed, n_new, n_destr) in enumerate(evals):
        if e:
            st.ResetPlan()
        st.SetJob(job)
        place = [(tgs[0], own[(e * 7 + k) % len(own)]) for k in range(n_destr)] + \
                [(tgs[k % len(tgs)], None) for k in range(n_new)]
        seqs.append(compute_placements(_Raw(), Plan(), job, place, synth.shuffle(len(nodes), seed), row_of,
                                       config is not None, direct=_Direct(st), eval_no=e))
        el = st.Eligibility()
        el.pop("escaped")
        eligs.append(el)
    return seqs, eligs


def _two_group_spread_job(nodes, n_own):
    import dataclasses
    from nomad_amd.structs import Spread, SpreadTarget, Task, TaskGroup
    base = synth.job_c2(200)
    web = dataclasses.replace(base.task_groups[0],
                              spreads=[Spread("${attr.kernel.name}", 60, [SpreadTarget("linux", 80)])])
    api = TaskGroup(name="api", count=200, ephemeral_disk_mb=150,
                    spreads=[Spread("${node.datacenter}", 30, [SpreadTarget("dc1", 100)])],
                    tasks=[Task(name="api", driver="exec", cpu=300, memory_mb=200)])
    return dataclasses.replace(base, task_groups=[web, api])


FB_EVALS = [(111, 60, 10), (112, 45, 20)]


@pytest.mark.parametrize("two_groups", [False, True])
def test_fallback_handoff_on_oracle(two_groups):
    nodes, allocs, job, tg = _cluster(900, 75, 60)
    tgs = [tg]
    if two_groups:
        job = _two_group_spread_job(nodes, 60)
        tgs = ["web", "api"]
    got, el_got, n_fb = _run_fb(lambda c: _FlakyOracle(c, 3), nodes, allocs, job, FB_EVALS, tgs)
    want, el_want = _direct_fb(nodes, allocs, job, FB_EVALS, tgs)
    assert n_fb > 20
    assert got == want
    assert el_got == el_want


@pytest.mark.gpu
@pytest.mark.parametrize("two_groups", [False, True])
def test_fallback_handoff_engine(monkeypatch, two_groups):
    """A mid-evaluation PE_EUNSUPPORTED (forced every 3rd Select): the Go chain
    answers with the engine's cursor, limit, spread groups and memo, and the
    engine continues from the chain's; placements and the final EvalEligibility
    equal the reference chain's driven call by call."""
    monkeypatch.setenv("PE_TEST_FALLBACK_EVERY", "3")
    nodes, allocs, job, tg = _cluster(2500, 76, 120)
    tgs = [tg]
    if two_groups:
        job = _two_group_spread_job(nodes, 120)
        tgs = ["web", "api"]
    got, el_got, n_fb = _run_fb(_engine, nodes, allocs, job, FB_EVALS, tgs)
    want, el_want = _direct_fb(nodes, allocs, job, FB_EVALS, tgs)
    assert n_fb > 20
    assert got == want
    assert el_got == el_want


@pytest.mark.gpu
def test_eligibility_mirror_behind_the_shim():
    """Without fallbacks, the shim's per-Select mirror of the engine's memo
    deltas equals the reference chain's ctx.Eligibility() after each eval."""
    nodes, allocs, job, tg = _cluster(3000, 77, 200)
    got, el_got, n_fb = _run_fb(_engine, nodes, allocs, job, EVALS, [tg])
    want, el_want = _direct_fb(nodes, allocs, job, EVALS, [tg])
    assert n_fb == 0
    assert got == want
    assert el_got == el_want


def _interleaved(make_stack, nodes, allocs, job, tg, config=None):
    """In-place updates on several nodes appended before the first Select
    (several AppendAllocs between two stack calls, across nodes), then fresh
    placements."""
    st = make_stack(config)
    st.SetState(nodes, allocs)
    shim = DeviceStack(st, Plan())
    shim.SetJob(job)
    own = [i for i, a in enumerate(allocs) if a.job_id == job.id]
    shim.SetNodes(synth.shuffle(len(nodes), 9))
    for k, a in enumerate(own[:25][::-1]):           # reverse node order on purpose
        shim.plan.AppendStoppedAlloc(a, st.row(allocs[a].node_id))
        shim.plan.AppendAlloc(PlanAlloc(id="u%d" % k, node_row=st.row(allocs[a].node_id), task_group=tg))
    out = []
    for i in range(80):
        r = shim.Select(tg)
        out.append(_key(r))
        if r is None:
            break
        shim.plan.AppendAlloc(PlanAlloc(id="p%d" % i, node_row=r.row, task_group=tg))
    return out


def test_interleaved_plan_appends_on_oracle():
    nodes, allocs, job, tg = _cluster(800, 78, 60)
    a = _interleaved(_oracle, nodes, allocs, job, tg)
    assert len(a) == 80


@pytest.mark.gpu
def test_interleaved_plan_appends_engine():
    nodes, allocs, job, tg = _cluster(800, 78, 60)
    assert _interleaved(_engine, nodes, allocs, job, tg) == _interleaved(_oracle, nodes, allocs, job, tg)
