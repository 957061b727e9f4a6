"""Zero-crossing served Selects (pe_spec_view, nomad_pe.h):
the caller answers plain Select / Commit pairs of computePlacements' loop
(generic_sched.go:552-627) from the engine's record view and calls C only
when it deviates. Every Select result, the cursor and the plan must equal the
oracle's one-at-a-time chain, with and without deviations, and the engine
must take the caller's counters over on its next entry point."""
import ctypes as C

import numpy as np
import pytest

from nomad_amd import abi, synth
from nomad_amd.stack import SelectOptions
from nomad_amd.structs import Job, Task, TaskGroup
from oracle.oracle import OracleGenericStack
from tests.test_dropin import _key, assert_equal_runs, compute_placements

pytestmark = pytest.mark.gpu


def _view(st):
    fn = st._lib.pe_spec_view_get
    fn.restype = C.POINTER(abi.pe_spec_view)
    fn.argtypes = [C.c_void_p]
    return fn(st._h).contents


def _rec_key(r, pre=()):
    return (r.row, r.final_score, tuple(r.scores[i] for i in range(r.n_scores)), r.nodes_evaluated,
            r.nodes_filtered, r.nodes_exhausted, r.new_offset, tuple(pre),
            tuple(r.device_offer_group[i] for i in range(r.n_device_offers)))


class ViewCaller:
    """The Go shim's fast path over an engine stack: Selects (plain, and the
    Preempt retry of a served nil) and the matching Commits from the view,
    everything else through C. The Commit of a record pe_select returned
    (the one that started a run) is confirmed through the view too, as
    nomad_pe.h allows."""

    def __init__(self, st):
        self.st = st
        self.v = _view(st)
        self.served = 0

    def _pre(self, k):
        v = self.v
        if not v.pre_off:
            return ()
        return tuple(v.pre_allocs[i] for i in range(v.pre_off[k], v.pre_off[k + 1]))

    def Select(self, tg, options=None):
        v = self.v
        plain = options is None or (not options.penalty_node_ids and not options.preferred_nodes)
        pre = bool(options is not None and options.preempt)
        if (plain and v.n_rec and v.tg_index == tg and v.served == v.confirmed and v.served < v.n_rec
                and bool(v.recs[v.served].flags & abi.PE_SPEC_PREEMPT) == pre):
            k = v.served
            r = v.recs[k]
            v.served += 1
            self.served += 1
            if r.row < 0:
                v.confirmed += 1   # a nil is settled at once
                return None
            return ("view", _rec_key(r, self._pre(k)))
        return self.st.Select(tg, options)

    def Commit(self, tg, row, preempted=()):
        v = self.v
        if (v.n_rec and v.tg_index == tg and v.served == v.confirmed + 1 and v.recs[v.served - 1].row == row
                and tuple(preempted) == self._pre(v.served - 1)):
            v.confirmed += 1
            return
        self.st.Commit(tg, row, preempted)


def view_placements(vc, count, preempt=False, tg=0, deviate=None, double_select=()):
    out = []

    def key(o):
        if o is None:
            return None
        return o[1] if isinstance(o, tuple) else _key(o)

    def row_of(o):
        return o[1][0] if isinstance(o, tuple) else o.row

    for i in range(count):
        if i in double_select:
            out.append(key(vc.Select(tg)))
        opt = vc.Select(tg)
        if opt is None and preempt:
            opt = vc.Select(tg, SelectOptions(preempt=True))
        out.append(key(opt))
        if opt is None:
            break
        row = row_of(opt)
        alt = deviate(i, opt) if deviate else None
        if alt is not None and alt != row:
            vc.Commit(tg, alt)
        else:
            vc.Commit(tg, row, opt[1][7] if isinstance(opt, tuple) else opt.preempted)
    return out


def _pair(nodes, allocs, job, perm):
    from nomad_amd.stack import GenericStack
    eng, ora = GenericStack(), OracleGenericStack()
    for st in (eng, ora):
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
    return eng, ora


@pytest.mark.parametrize("n,count", [(10000, 1000), (100, 10), (3000, 400)])
def test_view_serves_the_count_loop(n, count):
    nodes, allocs = synth.cluster_c2(n, seed=n)
    job = synth.job_c2(count) if n > 100 else synth.mock_job(count=count)
    perm = synth.shuffle(n, 2)
    eng, ora = _pair(nodes, allocs, job, perm)
    vc = ViewCaller(eng)
    a = view_placements(vc, count)
    b = compute_placements(ora, count)
    assert_equal_runs(a, b)
    assert vc.served >= count - 2   # everything after the first Select from the view
    off_e, off_o = (C.c_uint32(), C.c_uint32()), (C.c_uint32(), C.c_uint32())
    eng._lib.pe_get_cursor(C.c_void_p(eng._h), C.byref(off_e[0]), C.byref(off_e[1]))
    ora._lib.oracle_get_cursor(C.c_void_p(ora._h), C.byref(off_o[0]), C.byref(off_o[1]))
    assert (off_e[0].value, off_e[1].value) == (off_o[0].value, off_o[1].value)


def test_view_deviations():
    """Another row committed, a Select whose option is dropped, and a Preempt
    retry cross into C; the records after them still match the oracle."""
    nodes, allocs = synth.cluster_c2(4000, seed=9)
    job = synth.job_c2(300)
    perm = synth.shuffle(4000, 3)
    dev = lambda i, o: (perm[(i * 7) % 4000] if i % 37 == 5 else None)
    eng, ora = _pair(nodes, allocs, job, perm)
    a = view_placements(ViewCaller(eng), 300, deviate=dev, double_select=(11, 150))
    b = compute_placements(ora, 300, deviate=dev, double_select=(11, 150))
    assert_equal_runs(a, b)


def test_view_then_set_job_and_second_evaluation():
    """Counters taken over by SetJob / ResetPlan: a second evaluation on the
    same handle starts from the state the served commits left."""
    nodes, allocs = synth.cluster_c2(5000, seed=4)
    j1, j2 = synth.job_c2(200), synth.job_c2(150)
    j2.id = "second"
    perm = synth.shuffle(5000, 5)
    eng, ora = _pair(nodes, allocs, j1, perm)
    vc = ViewCaller(eng)
    a1 = view_placements(vc, 200)
    b1 = compute_placements(ora, 200)
    for st in (eng, ora):
        st.SetJob(j2)
        st.SetNodes(perm)
    a2 = view_placements(vc, 150)
    b2 = compute_placements(ora, 150)
    assert_equal_runs(a1 + a2, b1 + b2)


def test_dropin_loop_with_and_without_view():
    """The C caller loop (tools/dropin.cpp) with the view on and off gives the
    same rows per evaluation as the oracle driven by the same loop."""
    from tools import dropin
    from nomad_amd.stack import GenericStack
    nodes, allocs = synth.cluster_c2(10000, seed=42)
    job = synth.job_c2(1000)
    orders = np.stack([np.asarray(synth.shuffle(10000, s), dtype=np.uint32) for s in (1, 2, 3)])
    rows = {}
    for mode in ("view", "cross", "oracle"):
        st = OracleGenericStack() if mode == "oracle" else GenericStack()
        st.SetState(nodes, allocs)
        dropin.use_view(mode == "view")
        dropin.view_served(reset=True)
        run = dropin.prepare(st, job)
        placed, evals, selects, secs, last = run(orders, 1000)
        rows[mode] = (placed, evals, list(last))
        if mode == "view":
            assert dropin.view_served() >= 3 * 990
        st.close()
    dropin.use_view(True)
    assert rows["view"] == rows["cross"] == rows["oracle"]


# ---- every Select answer, nils included (the Preempt retry protocol, §25) ----

def _nil_key(r):
    return ("nil", r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted, r.new_offset)


class CCaller:
    """Every Select and Commit through the stack's entry points (engine or oracle)."""

    def __init__(self, st):
        self.st = st

    def sel(self, tg, options=None):
        r = self.st.SelectRaw(tg, options)
        if r.row < 0:
            return _nil_key(r), -1, ()
        return _key(r), r.row, tuple(r.preempted)

    def commit(self, tg, row, pre=()):
        self.st.Commit(tg, row, pre)


class ViewAnswers(ViewCaller):
    """ViewCaller answering with the full record key, nils included."""

    def sel(self, tg, options=None):
        v = self.v
        pre = bool(options is not None and options.preempt)
        if (v.n_rec and v.tg_index == tg and v.served == v.confirmed and v.served < v.n_rec
                and bool(v.recs[v.served].flags & abi.PE_SPEC_PREEMPT) == pre):
            k = v.served
            r = v.recs[k]
            v.served += 1
            self.served += 1
            if r.row < 0:
                v.confirmed += 1
                return _nil_key(r), -1, ()
            p = self._pre(k)
            return _rec_key(r, p), r.row, p
        return CCaller(self.st).sel(tg, options)

    def commit(self, tg, row, pre=()):
        self.Commit(tg, row, pre)


def protocol_answers(caller, count, preempt=True, tg=0, deviate=None):
    """computePlacements' loop (generic_sched.go:552-627, 773-792) recording
    every Select answer. deviate(i, row) -> a row to commit instead (its
    preemptions dropped), or None."""
    out = []
    for i in range(count):
        k, row, pre = caller.sel(tg)
        out.append(k)
        if row < 0 and preempt:
            k, row, pre = caller.sel(tg, SelectOptions(preempt=True))
            out.append(k)
        if row < 0:
            break
        alt = deviate(i, row) if deviate else None
        if alt is not None and alt != row:
            caller.commit(tg, alt)
        else:
            caller.commit(tg, row, pre)
    return out


def _c5_pair(n, busy, count, seed=5, perm_seed=77):
    from nomad_amd.stack import GenericStack
    from nomad_amd.structs import SchedulerConfig
    nodes, allocs = synth.cluster_c5(n, seed=seed, busy=busy)
    job = synth.job_c5(count)
    perm = synth.shuffle(n, perm_seed)
    cfg = SchedulerConfig(preempt_service=True)
    eng, ora = GenericStack(config=cfg), OracleGenericStack(config=cfg)
    for st in (eng, ora):
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
    return eng, ora, perm


@pytest.mark.parametrize("n,busy,count", [(800, 0.9, 120), (5000, 0.99, 300)])
def test_view_serves_the_preempt_retry(n, busy, count):
    """Plain nils, Preempt options with their PreemptedAllocs and the commits
    that name them, all from the view; equal to the oracle answer by answer."""
    eng, ora, _ = _c5_pair(n, busy, count)
    vc = ViewAnswers(eng)
    a = protocol_answers(vc, count)
    b = protocol_answers(CCaller(ora), count)
    assert_equal_runs(a, b)
    assert sum(1 for x in b if x[0] != "nil" and x[7]) >= 10, "too few evicting placements"
    assert vc.served >= len(a) - 12, (vc.served, len(a))
    assert eng.SpeculationStats()[2] == 0   # no rollback


def test_c_path_serves_the_preempt_retry():
    """The same records through pe_select / pe_commit_preempt (no view)."""
    eng, ora, _ = _c5_pair(800, 0.9, 120, seed=6)
    a = protocol_answers(CCaller(eng), 120)
    b = protocol_answers(CCaller(ora), 120)
    assert_equal_runs(a, b)
    runs, served, rollbacks, _ = eng.SpeculationStats()
    assert served >= len(a) - 20 and rollbacks == 0, eng.SpeculationStats()


@pytest.mark.parametrize("via_view", [True, False])
def test_preempt_retry_deviations(via_view):
    """Commits of another row (an evicting placement's preemptions dropped)
    roll the run back to its confirmed prefix: evictions, preempted flags and
    the plan's preemption counts included."""
    eng, ora, perm = _c5_pair(1500, 0.97, 200, seed=8)
    dev = lambda i, row: (int(perm[(i * 13) % len(perm)]) if i % 29 == 7 else None)
    a = protocol_answers(ViewAnswers(eng) if via_view else CCaller(eng), 200, deviate=dev)
    b = protocol_answers(CCaller(ora), 200, deviate=dev)
    assert_equal_runs(a, b)
    assert eng.SpeculationStats()[2] >= 3


def test_view_confirms_a_record_pe_select_returned():
    """nomad_pe.h lets the caller confirm, through the view, the record the
    run's first pe_select returned; the engine's plan mirror must then hold
    that placement: a job-level distinct_property makes the second task
    group's Selects read it (propertyset.go:54-114)."""
    from nomad_amd.stack import GenericStack
    from nomad_amd.structs import Constraint
    nodes = []
    for i in range(240):
        nd = synth.mock_node("node-%d" % i)
        nd.meta["rack"] = "r%d" % (i % 48)
        nd.compute_class()
        nodes.append(nd)

    def tg(name, count):
        return TaskGroup(name=name, count=count, ephemeral_disk_mb=0,
                         tasks=[Task(name="web", driver="exec", cpu=100, memory_mb=64)])
    job = Job(id="dp", constraints=[Constraint("${meta.rack}", "", "distinct_property")],
              task_groups=[tg("bar", 30), tg("baz", 12)])
    perm = synth.shuffle(len(nodes), 3)
    eng, ora = GenericStack(), OracleGenericStack()
    for st in (eng, ora):
        st.SetState(nodes, [])
        st.SetJob(job)
        st.SetNodes(perm)
    vc = ViewAnswers(eng)
    a = protocol_answers(vc, 30, preempt=False, tg=0) + protocol_answers(vc, 12, preempt=False, tg=1)
    b = protocol_answers(CCaller(ora), 30, preempt=False, tg=0) + \
        protocol_answers(CCaller(ora), 12, preempt=False, tg=1)
    assert_equal_runs(a, b)
    assert vc.served >= 20
