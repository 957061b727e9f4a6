"""AllocMetric maps of Select: ClassFiltered,
ConstraintFiltered, ClassExhausted, DimensionExhausted
(nomad/structs/structs.go:9903-9937) and ScoreMetaData (ScoreNode +
PopulateScoreMetaData over the top-5 kheap, structs.go:9976-10018,
lib/kheap/score_heap.go), as `ctx.Metrics()` holds them after
GenericStack.Select.

KATs follow the reference's own assertions (stack_test.go:310-348
TestServiceStack_Select_ConstraintFilter, :350-392
TestServiceStack_Select_BinPack_Overflow) on the oracle and the engine. The
GPU tests then compare the engine's maps with the oracle's Select by Select
over count loops that filter (class memo, escaped constraints, drivers,
distinct_hosts, distinct_property) and exhaust (cpu, memory, network,
devices), windowed and full-pass.
"""
import pytest

from nomad_amd import synth
from nomad_amd.structs import Allocation, Constraint, Job, NetworkResource, Task, TaskGroup
from oracle.oracle import OracleGenericStack


def _engine():
    from nomad_amd.stack import GenericStack
    return GenericStack()


STACKS = [pytest.param(OracleGenericStack, id="oracle"),
          pytest.param(_engine, id="engine", marks=pytest.mark.gpu)]


def _mk(stack_cls, nodes, allocs, job):
    st = stack_cls()
    st.EnableMetrics()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    return st


@pytest.mark.parametrize("stack_cls", STACKS)
def test_constraint_filter_kat(stack_cls):
    nodes = [synth.mock_node("a"), synth.mock_node("b")]
    nodes[0].attributes["kernel.name"] = "freebsd"
    nodes[0].compute_class()
    job = synth.mock_job()
    job.constraints[0].rtarget = "freebsd"
    st = _mk(stack_cls, nodes, [], job)
    st.SetNodes(nodes)
    r = st.SelectRaw(0)
    assert r.row == 0 and r.nodes_filtered == 1
    m = st.LastMetrics()
    assert m["ClassFiltered"] == {"linux-medium-pci": 1}
    assert m["ConstraintFiltered"] == {"${attr.kernel.name} = freebsd": 1}
    assert m["ClassExhausted"] == {} and m["DimensionExhausted"] == {}


@pytest.mark.parametrize("stack_cls", STACKS)
def test_binpack_overflow_kat(stack_cls):
    nodes = [synth.mock_node("a"), synth.mock_node("b")]
    nodes[1].reserved_cpu = nodes[1].cpu_shares
    nodes[1].reserved_memory_mb = nodes[1].reserved_disk_mb = 0
    st = _mk(stack_cls, nodes, [], synth.mock_job())
    st.SetNodes(nodes)
    r = st.SelectRaw(0)
    assert r.row == 0 and r.nodes_exhausted == 1
    m = st.LastMetrics()
    assert m["ClassExhausted"] == {"linux-medium-pci": 1}
    assert m["DimensionExhausted"] == {"cpu": 1}
    # "Expect score metadata for one node" (PopulateScoreMetaData, top 5 by NormScore)
    assert len(m["ScoreMetaData"]) == 1
    node_id, norm, scores = m["ScoreMetaData"][0]
    assert node_id == "a" and norm == r.final_score
    assert set(scores) == {"binpack", "job-anti-affinity", "node-reschedule-penalty", "node-affinity"}
    assert scores["binpack"] == r.scores[0] and scores["node-affinity"] == 0.0


def _loop(nodes, allocs, job, perm, placements, tg=0):
    """Select + Commit on both sides; every Select's result and maps equal."""
    from nomad_amd.stack import GenericStack
    sts = []
    for cls in (GenericStack, OracleGenericStack):
        st = cls()
        st.EnableMetrics()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
        sts.append(st)
    eng, ora = sts
    seen = {"ConstraintFiltered": set(), "DimensionExhausted": set()}
    for k in range(placements):
        re, ro = eng.SelectRaw(tg), ora.SelectRaw(tg)
        assert (re.row, re.nodes_evaluated, re.nodes_filtered, re.nodes_exhausted) == \
            (ro.row, ro.nodes_evaluated, ro.nodes_filtered, ro.nodes_exhausted), k
        me, mo = eng.LastMetrics(), ora.LastMetrics()
        assert me == mo, (k, me, mo)
        for key in seen:
            seen[key] |= set(mo[key])
        if ro.row < 0:
            break
        eng.Commit(tg, re.row)
        ora.Commit(tg, ro.row)
    return seen


@pytest.mark.gpu
def test_metrics_windowed_count_loop():
    # C2-shaped: heterogeneous nodes, class-memo filtering and cpu/memory exhaustion
    nodes, allocs = synth.cluster_c2(600, seed=3)
    for i, nd in enumerate(nodes):
        if i % 7 == 0:
            nd.attributes["kernel.name"] = "windows"
            nd.compute_class()
        if i % 11 == 0:
            nd.drivers = {}
            nd.attributes.pop("driver.exec", None)
            nd.compute_class()
    job = synth.job_c2(400)
    job.constraints.append(Constraint("${attr.kernel.name}", "linux", "="))
    job.task_groups[0].tasks[0].cpu = 2500
    job.task_groups[0].tasks[0].memory_mb = 6000
    seen = _loop(nodes, allocs, job, synth.shuffle(len(nodes), 9), 400)
    assert "${attr.kernel.name} = linux" in seen["ConstraintFiltered"]
    assert "missing drivers" in seen["ConstraintFiltered"]
    assert "computed class ineligible" in seen["ConstraintFiltered"]
    assert seen["DimensionExhausted"] & {"cpu", "memory"}


@pytest.mark.gpu
def test_metrics_full_pass_spread_affinity():
    # C3-shaped: semver / regexp constraints, affinity + spread (limit MaxInt32)
    nodes, allocs = synth.cluster_c3(1500, seed=8)
    seen = _loop(nodes, allocs, synth.job_c3(60), synth.shuffle(len(nodes), 2), 60)
    assert len(seen["ConstraintFiltered"]) >= 2


@pytest.mark.gpu
def test_metrics_escaped_and_distinct():
    # escaped constraint (${node.unique.id}) runs per node; distinct_hosts and
    # distinct_property filter after the wrapper
    nodes, allocs = synth.cluster_c3(400, seed=4)
    job = synth.job_c2(120)
    job.constraints.append(Constraint("${meta.rack}", "3", "distinct_property"))
    job.task_groups[0].constraints.append(Constraint("${node.unique.id}", nodes[5].id, "!="))
    job.task_groups[0].constraints.append(Constraint("", "", "distinct_hosts"))
    seen = _loop(nodes, allocs, job, synth.shuffle(len(nodes), 6), 120)
    assert "distinct_hosts" in seen["ConstraintFiltered"]
    assert any(k.startswith("distinct_property: ${meta.rack}=") for k in seen["ConstraintFiltered"])


@pytest.mark.gpu
def test_metrics_network_and_devices():
    nodes, allocs = synth.cluster_c5(800, seed=5, busy=0.5)
    job = synth.job_c5(150)
    seen = _loop(nodes, allocs, job, synth.shuffle(len(nodes), 3), 150)
    assert any(k.startswith("devices: ") for k in seen["DimensionExhausted"]) or \
        "missing devices" in seen["ConstraintFiltered"]
    # bandwidth: a task network ask larger than what the nodes have left
    nodes2, allocs2 = synth.cluster_c2(300, seed=2)
    job2 = synth.job_c2(100)
    job2.task_groups[0].tasks[0].network = NetworkResource(mbits=400)
    seen2 = _loop(nodes2, allocs2, job2, synth.shuffle(len(nodes2), 4), 100)
    assert any(k.startswith("network: ") for k in seen2["DimensionExhausted"])


@pytest.mark.gpu
def test_metrics_preferred_and_penalty_nodes():
    # SelectOptions: PreferredNodes (inner Select over them first, its own
    # AllocMetric) and PenaltyNodeIDs (node-reschedule-penalty score of -1)
    import random
    from nomad_amd.stack import GenericStack, SelectOptions
    nodes, allocs = synth.cluster_c2(300, seed=5)
    job = synth.job_c2(90)
    perm = synth.shuffle(len(nodes), 8)
    rng = random.Random(3)
    sts = []
    for cls in (GenericStack, OracleGenericStack):
        st = cls()
        st.EnableMetrics()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
        sts.append(st)
    eng, ora = sts
    for k in range(90):
        opt = None
        if k % 3 == 0:
            opt = SelectOptions(preferred_nodes=[n.id for n in rng.sample(nodes, 3)],
                                penalty_node_ids=[n.id for n in rng.sample(nodes, 40)])
        elif k % 3 == 1:
            opt = SelectOptions(penalty_node_ids=[n.id for n in rng.sample(nodes, 40)])
        re, ro = eng.Select(0, opt), ora.Select(0, opt)
        assert (re.row if re else -1) == (ro.row if ro else -1), k
        assert eng.LastMetrics() == ora.LastMetrics(), k
        if ro is None:
            break
        eng.Commit(0, re.row)
        ora.Commit(0, ro.row)


@pytest.mark.gpu
def test_metrics_system_stack():
    # SystemScheduler: one single-node Select per node (SetNodes([node])); the
    # SystemStack ranks with BinPack alone, so ScoreMetaData holds binpack and
    # normalized-score only (stack.go:277-281)
    from nomad_amd.stack import SystemStack
    from oracle.oracle import OracleSystemStack
    nodes, allocs = synth.cluster_c4(300, seed=13)
    job = synth.mock_system_job()
    sts = []
    for cls in (SystemStack, OracleSystemStack):
        st = cls()
        st.EnableMetrics()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        sts.append(st)
    eng, ora = sts
    seen = set()
    for nd in nodes:
        eng.SetNodes([nd])
        ora.SetNodes([nd])
        re, ro = eng.SelectRaw(0), ora.SelectRaw(0)
        assert (re.row, re.nodes_filtered, re.nodes_exhausted) == (ro.row, ro.nodes_filtered, ro.nodes_exhausted)
        me, mo = eng.LastMetrics(), ora.LastMetrics()
        assert me == mo, (nd.id, me, mo)
        seen |= set(mo["ConstraintFiltered"]) | set(mo["DimensionExhausted"])
        if ro.row >= 0:
            assert set(mo["ScoreMetaData"][0][2]) <= {"binpack", "devices"}
            eng.Commit(0, re.row)
            ora.Commit(0, ro.row)
    assert seen


def _preempt_loop(nodes, allocs, job, perm, placements, config, system=False):
    """computePlacements with selectNextOption's Preempt retry (generic_sched.go:
    773-792): every Select's maps equal, the Preempt ones included (BinPack with
    evict: ExhaustedNode when no preemption frees enough, rank.go:480-503;
    ScoreNode("preemption"), rank.go:793-806)."""
    from nomad_amd.stack import GenericStack, SelectOptions
    sts = []
    for cls in (GenericStack, OracleGenericStack):
        st = cls(config=config)
        st.EnableMetrics()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
        sts.append(st)
    eng, ora = sts
    seen = {"preemption": 0, "exhausted": set()}
    for k in range(placements):
        for opts in (None, SelectOptions(preempt=True)):
            re, ro = eng.SelectRaw(0, opts), ora.SelectRaw(0, opts)
            assert (re.row, re.nodes_evaluated, re.nodes_filtered, re.nodes_exhausted, re.preempted) == \
                (ro.row, ro.nodes_evaluated, ro.nodes_filtered, ro.nodes_exhausted, ro.preempted), (k, opts)
            me, mo = eng.LastMetrics(), ora.LastMetrics()
            assert me == mo, (k, opts, me, mo)
            seen["exhausted"] |= set(mo["DimensionExhausted"])
            seen["preemption"] += sum(1 for x in mo["ScoreMetaData"] if "preemption" in x[2])
            if ro.row >= 0:
                break
        if ro.row < 0:
            break
        eng.Commit(0, re.row, re.preempted)
        ora.Commit(0, ro.row, ro.preempted)
    return seen


@pytest.mark.gpu
def test_metrics_preempt_selects():
    from nomad_amd.structs import SchedulerConfig
    nodes, allocs = synth.cluster_c5(700, seed=21, busy=0.95)
    job = synth.job_c5(120)
    seen = _preempt_loop(nodes, allocs, job, synth.shuffle(len(nodes), 4), 120,
                         SchedulerConfig(preempt_service=True))
    assert seen["preemption"] > 0


@pytest.mark.gpu
def test_metrics_preempt_selects_cpu_memory():
    # no devices: PreemptForTaskGroup frees cpu / memory; nodes where it cannot
    # are ExhaustedNode(dim)
    from nomad_amd.structs import Allocation, SchedulerConfig
    nodes, allocs = synth.cluster_c2(500, seed=22)
    for i, nd in enumerate(nodes):
        allocs.append(Allocation(node_id=nd.id, job_id="low-%d" % (i % 5), task_group="tg",
                                 cpu_shares=max(0, nd.cpu_shares - 100 - 600 - (i % 3) * 200), memory_mb=64,
                                 disk_mb=10, priority=10 + (i % 4) * 10))
    job = synth.job_c2(200)
    job.priority = 70
    seen = _preempt_loop(nodes, allocs, job, synth.shuffle(len(nodes), 5), 200,
                         SchedulerConfig(preempt_service=True))
    assert seen["preemption"] > 0


def _view_metrics_loop(nodes, allocs, job, perm, placements, tg=0, deviate=()):
    """The Go shim's zero-crossing path with metrics on: Selects and Commits
    from the served-Select view, each served record's maps read from the view
    (pe_spec_view.mcounts / mscores, binary), the rest through C (both the
    text and the binary maps); every Select's result and maps equal the
    oracle's (generic_sched.go:558, 587: Allocation.Metrics)."""
    import ctypes as C
    from nomad_amd import abi
    from nomad_amd.stack import GenericStack, view_metrics
    eng, ora = GenericStack(), OracleGenericStack()
    for st in (eng, ora):
        st.EnableMetrics()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
    fn = eng._lib.pe_spec_view_get
    fn.restype = C.POINTER(abi.pe_spec_view)
    fn.argtypes = [C.c_void_p]
    v = fn(eng._h).contents
    from_view = 0
    for k in range(placements):
        ro = ora.SelectRaw(tg)
        mo = ora.LastMetrics()
        if v.n_rec and v.tg_index == tg and v.served == v.confirmed and v.served < v.n_rec:
            assert v.mcounts_off and v.mscores_off, "served records carry no maps"
            i = v.served
            r = v.recs[i]
            me = view_metrics(eng, v, i)
            v.served += 1
            if r.row < 0:
                v.confirmed += 1
            from_view += 1
            got = (r.row, r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted)
        else:
            re = eng.SelectRaw(tg)
            me = eng.LastMetrics()
            assert eng.LastMetricsBin() == me, k
            got = (re.row, re.nodes_evaluated, re.nodes_filtered, re.nodes_exhausted)
        assert got == (ro.row, ro.nodes_evaluated, ro.nodes_filtered, ro.nodes_exhausted), k
        assert me == mo, (k, me, mo)
        if ro.row < 0:
            break
        row = ro.row
        if k in deviate:   # another row: the run is rolled back, the memo rewound
            row = int(perm[(k * 31) % len(perm)])
        if k not in deviate and v.n_rec and v.tg_index == tg and v.served == v.confirmed + 1 \
                and v.recs[v.served - 1].row == row:
            v.confirmed += 1
        else:
            eng.Commit(tg, row)
        ora.Commit(tg, row)
    return from_view, eng


@pytest.mark.gpu
@pytest.mark.parametrize("deviate", [(), (3, 4, 57, 120)])
def test_metrics_served_from_the_view(deviate):
    nodes, allocs = synth.cluster_c2(600, seed=3)
    for i, nd in enumerate(nodes):
        if i % 7 == 0:
            nd.attributes["kernel.name"] = "windows"
            nd.compute_class()
        if i % 11 == 0:
            nd.drivers = {}
            nd.attributes.pop("driver.exec", None)
            nd.compute_class()
    job = synth.job_c2(300)
    job.constraints.append(Constraint("${attr.kernel.name}", "linux", "="))
    job.task_groups[0].tasks[0].cpu = 2500
    job.task_groups[0].tasks[0].memory_mb = 6000
    from_view, eng = _view_metrics_loop(nodes, allocs, job, synth.shuffle(len(nodes), 9), 300, deviate=deviate)
    assert from_view >= 250, from_view
    runs, served, rollbacks, _ = eng.SpeculationStats()
    assert runs >= 1 and rollbacks >= (1 if deviate else 0), eng.SpeculationStats()


@pytest.mark.gpu
def test_metrics_served_from_the_view_devices():
    # device asks: the traced rows' free instances after the earlier records' offers
    nodes, allocs = synth.cluster_c5(900, seed=4, busy=0.3)
    job = synth.job_c5(150)
    from_view, _ = _view_metrics_loop(nodes, allocs, job, synth.shuffle(len(nodes), 5), 150)
    assert from_view >= 100, from_view


def _view_metrics_protocol(eng, ora, count, preempt=False, tg=0, deviate=None):
    """computePlacements' loop (Select, the Preempt retry on nil when
    preemption is on, Commit with the preempted set) with AllocMetric on:
    every Select answered from the served-Select view when it can be (its
    maps from the view's binary arrays), else through C; every answer and
    its maps equal the oracle's. deviate(i, row) -> another row to commit."""
    import ctypes as C
    from nomad_amd import abi
    from nomad_amd.stack import SelectOptions, view_metrics
    from tests.test_dropin import _key
    from tests.test_spec_view import _rec_key
    fn = eng._lib.pe_spec_view_get
    fn.restype = C.POINTER(abi.pe_spec_view)
    fn.argtypes = [C.c_void_p]
    v = fn(eng._h).contents
    stats = {"view": 0, "c": 0, "evicting": 0}

    def ora_sel(opts):
        r = ora.SelectRaw(tg, opts)
        return (_key(r) if r.row >= 0 else ("nil", r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted,
                                            r.new_offset)), r.row, tuple(r.preempted), ora.LastMetrics()

    def eng_sel(opts):
        pre = bool(opts is not None and opts.preempt)
        if (v.n_rec and v.tg_index == tg and v.served == v.confirmed and v.served < v.n_rec
                and bool(v.recs[v.served].flags & abi.PE_SPEC_PREEMPT) == pre):
            assert v.mcounts_off and v.mscores_off, "served records carry no maps"
            k = v.served
            r = v.recs[k]
            m = view_metrics(eng, v, k)
            v.served += 1
            stats["view"] += 1
            p = tuple(v.pre_allocs[i] for i in range(v.pre_off[k], v.pre_off[k + 1])) if v.pre_off else ()
            if r.row < 0:
                v.confirmed += 1
                return ("nil", r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted, r.new_offset), -1, (), m
            return _rec_key(r, p), r.row, p, m
        stats["c"] += 1
        r = eng.SelectRaw(tg, opts)
        m = eng.LastMetricsBin()
        assert m == eng.LastMetrics()
        return (_key(r) if r.row >= 0 else ("nil", r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted,
                                            r.new_offset)), r.row, tuple(r.preempted), m

    def eng_commit(row, pre):
        if (v.n_rec and v.tg_index == tg and v.served == v.confirmed + 1 and v.recs[v.served - 1].row == row
                and tuple(pre) == (tuple(v.pre_allocs[i] for i in range(v.pre_off[v.served - 1],
                                                                       v.pre_off[v.served]))
                                   if v.pre_off else ())):
            v.confirmed += 1
        else:
            eng.Commit(tg, row, pre)

    answers = 0
    for i in range(count):
        for opts in ((None, SelectOptions(preempt=True)) if preempt else (None,)):
            ke, re_, pe_, me = eng_sel(opts)
            ko, ro, po, mo = ora_sel(opts)
            answers += 1
            assert ke[:7] == ko[:7] and pe_ == po, ("answer %d" % answers, ke, ko)
            assert me == mo, ("answer %d maps" % answers, me, mo)
            if ro >= 0:
                break
        if ro < 0:
            break
        stats["evicting"] += bool(po)
        alt = deviate(i, ro) if deviate else None
        if alt is not None and alt != ro:
            eng_commit(alt, ())
            ora.Commit(tg, alt)
        else:
            eng_commit(ro, po)
            ora.Commit(tg, ro, po)
    return stats


def _metrics_pair(nodes, allocs, job, perm, config=None):
    from nomad_amd.stack import GenericStack
    eng, ora = GenericStack(config=config), OracleGenericStack(config=config)
    for st in (eng, ora):
        st.EnableMetrics()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
    return eng, ora


@pytest.mark.gpu
def test_metrics_view_c3_full_scan():
    """C3 at its bench shape (10k nodes, spread + affinity + semver/regexp):
    full-pass runs with AllocMetric on, every record's maps from the view."""
    nodes, allocs = synth.cluster_c3(10000, seed=7)
    eng, ora = _metrics_pair(nodes, allocs, synth.job_c3(300), synth.shuffle(10000, 17))
    st = _view_metrics_protocol(eng, ora, 300)
    assert st["view"] >= 280, st


@pytest.mark.gpu
@pytest.mark.parametrize("dev", [False, True])
def test_metrics_view_preempt_retry(dev):
    """Evicting runs (preemption on, a saturated C5-shaped cluster): the plain
    nils and the Preempt options with their maps (preemption scores
    included) from the view, with and without deviating commits."""
    from nomad_amd.structs import SchedulerConfig
    nodes, allocs = synth.cluster_c5(3000, seed=5, busy=0.97)
    perm = synth.shuffle(len(nodes), 77)
    eng, ora = _metrics_pair(nodes, allocs, synth.job_c5(250), perm, SchedulerConfig(preempt_service=True))
    deviate = (lambda i, row: int(perm[(i * 13) % len(perm)]) if i % 41 == 17 else None) if dev else None
    st = _view_metrics_protocol(eng, ora, 250, preempt=True, deviate=deviate)
    assert st["evicting"] >= 20 and st["view"] >= 200, st


@pytest.mark.gpu
def test_metrics_view_c5_bench_shape_prefix():
    """C5 at its bench shape (50k nodes, 99 % of the GPU nodes busy): the
    evaluation's first 400 placements (the free instances, then the first
    evicting placements), every answer's maps equal to the oracle's."""
    from nomad_amd.structs import SchedulerConfig
    nodes, allocs = synth.cluster_c5(50000, seed=5, busy=0.99)
    eng, ora = _metrics_pair(nodes, allocs, synth.job_c5(1000), synth.shuffle(50000, 77),
                             SchedulerConfig(preempt_service=True))
    st = _view_metrics_protocol(eng, ora, 400, preempt=True)
    assert st["evicting"] >= 10, st


@pytest.mark.gpu
def test_metrics_view_distinct_property_and_spread():
    """Property sets (a job-level distinct_property and a spread): replayed
    runs, maps from the view."""
    from nomad_amd.structs import Spread
    nodes, allocs = synth.cluster_c2(2000, seed=12)
    for i, nd in enumerate(nodes):
        nd.meta["rack"] = "r%d" % (i % 90)
        nd.compute_class()
    job = synth.job_c2(120)
    job.constraints.append(Constraint("${meta.rack}", "2", "distinct_property"))
    job.task_groups[0].spreads = [Spread("${node.datacenter}", 50, [])]
    eng, ora = _metrics_pair(nodes, allocs, job, synth.shuffle(len(nodes), 4))
    st = _view_metrics_protocol(eng, ora, 120)
    assert st["view"] >= 100, st


@pytest.mark.gpu
def test_metrics_system_c4_100k():
    """C4 at its bench shape (100k nodes): SystemScheduler's per-node
    SetNodes([node]) + Select + Commit with AllocMetric on, answered from the
    engine's per-row cache (one k_system pass plus one k_trace pass); every
    node's maps equal the oracle's, the memo's "computed class ineligible"
    included."""
    import numpy as np
    from nomad_amd import synth_columnar
    from nomad_amd.stack import SystemStack
    from oracle.oracle import OracleSystemStack
    n = 100000
    cs = synth_columnar.ColumnarState(n, seed=11, kind="c4", prefill=0.05)
    job = synth.mock_system_job()
    rows = np.random.Generator(np.random.PCG64(5)).permutation(n).astype(np.uint32)
    eng, ora = SystemStack(), OracleSystemStack()
    for st in (eng, ora):
        st.EnableMetrics()
        st.SetStateColumnar(cs)
        st.SetJob(job)
    kinds = set()
    for i, r in enumerate(rows):
        eng.SetNodes([int(r)])
        ora.SetNodes([int(r)])
        re, ro = eng.SelectRaw(0), ora.SelectRaw(0)
        assert (re.row, re.final_score, re.nodes_filtered, re.nodes_exhausted) == \
               (ro.row, ro.final_score, ro.nodes_filtered, ro.nodes_exhausted), i
        me, mo = eng.LastMetrics(), ora.LastMetrics()
        assert me == mo, (i, me, mo)
        if i % 997 == 0:
            assert eng.LastMetricsBin() == me, i
        kinds |= {k for k in ("ConstraintFiltered", "DimensionExhausted", "ScoreMetaData") if mo[k]}
        if ro.row >= 0:
            eng.Commit(0, re.row)
            ora.Commit(0, ro.row)
    assert kinds == {"ConstraintFiltered", "DimensionExhausted", "ScoreMetaData"}, kinds
    import ctypes as C
    out = (C.c_uint64 * 2)()
    eng._check(eng._lib.pe_system_spec_stats(C.c_void_p(eng._h), out))
    assert out[1] >= n - 2, tuple(out)   # every Select after the pass's first from the cache


@pytest.mark.gpu
def test_metrics_system_view_c4_100k():
    """The served system-Select view with AllocMetric on, at the C4 bench
    shape: the caller answers SetNodes([node]) + Select + Commit from the
    view and assembles each Select's maps from its per-row entries
    (pe_system_view.mkey / mclass / mfailed / mscore / mnode_class, as the Go
    shim would); every node's maps equal the oracle's, and a crossing Select
    afterwards (the log taken over: the memo and the last maps) too."""
    import ctypes as C
    import numpy as np
    from nomad_amd import abi, synth_columnar
    from nomad_amd.stack import SystemStack
    from oracle.oracle import OracleSystemStack
    n = 100000
    cs = synth_columnar.ColumnarState(n, seed=11, kind="c4", prefill=0.05)
    job = synth.mock_system_job()
    rows = np.random.Generator(np.random.PCG64(5)).permutation(n).astype(np.uint32)
    eng, ora = SystemStack(), OracleSystemStack()
    for st in (eng, ora):
        st.EnableMetrics()
        st.SetStateColumnar(cs)
        st.SetJob(job)
    fn = eng._lib.pe_system_view_get
    fn.restype = C.POINTER(abi.pe_system_view)
    fn.argtypes = [C.c_void_p]
    v = fn(eng._h).contents
    keys = {}

    def key(k):
        if k not in keys:
            keys[k] = eng.MetricString(k)
        return keys[k]

    def view_maps(r, code, score):
        m = {"ClassFiltered": {}, "ConstraintFiltered": {}, "ClassExhausted": {}, "DimensionExhausted": {},
             "ScoreMetaData": []}
        nc = v.mnode_class[r]
        if code == 0:
            m["ScoreMetaData"] = [(cs.node_id(r), score, {"binpack": v.mscore[r]})]
        elif code == 1:
            k, mc = v.mkey[r], v.mclass[r]
            if mc != abi.PE_NONE:
                if v.mfailed[mc]:
                    k = v.mkey_ineligible
                v.mfailed[mc] = 1
            if nc != abi.PE_NONE:
                m["ClassFiltered"] = {key(nc): 1}
            m["ConstraintFiltered"] = {key(k): 1}
        else:
            if nc != abi.PE_NONE:
                m["ClassExhausted"] = {key(nc): 1}
            m["DimensionExhausted"] = {key(v.mkey[r]): 1}
        return m

    served = 0
    for i, r in enumerate(rows):
        r = int(r)
        ora.SetNodes([r])
        ro = ora.SelectRaw(0)
        mo = ora.LastMetrics()
        bits = v.outcome[r] if v.n_rows else 0x7FF8000000000003
        nan = (bits & 0x7FF8000000000000) == 0x7FF8000000000000
        code = bits & 3 if nan else 0
        if not v.n_rows or r >= v.n_rows or code == 3 or v.n_log >= v.log_cap:
            eng.SetNodes([r])
            re = eng.SelectRaw(0)
            got = (re.row, re.final_score) if re.row >= 0 else None
            me = eng.LastMetrics()
            if re.row >= 0:
                eng.Commit(0, re.row)
        else:
            assert v.mkey and v.mfailed, "the view carries no metric entries"
            score = C.c_double.from_buffer_copy(C.c_uint64(bits)).value
            me = view_maps(r, code, score)
            if code:
                v.log[v.n_log] = r | abi.PE_SYS_NIL
                got = None
            else:
                v.log[v.n_log] = r | abi.PE_SYS_COMMITTED
                v.outcome[r] = abi.PE_SYS_STALE
                got = (r, score)
            v.n_log += 1
            served += 1
        assert got == ((ro.row, ro.final_score) if ro.row >= 0 else None), i
        assert me == mo, (i, me, mo)
        if ro.row >= 0:
            ora.Commit(0, ro.row)
        if i == 50000:   # a crossing in the middle: the log is taken over, the last maps with it
            assert eng.LastMetrics() == mo
    assert served >= n - 10, served


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["even_and_targets", "per_node_values", "affinity_only"])
def test_metrics_view_batched_spreads(kind):
    """Full-pass runs traced in one batch (spec_metrics): every record's spread
    boosts from its own use counts (k_spread_tables), an even spread beside a
    targeted one over 90 values, a spread over a per-node attribute, and an
    affinity-only full pass; maps from the view equal the oracle's."""
    from nomad_amd.structs import Affinity, Spread, SpreadTarget
    nodes, allocs = synth.cluster_c2(2000, seed=13)
    for i, nd in enumerate(nodes):
        nd.meta["rack"] = "r%d" % (i % 90)
        nd.datacenter = "dc%d" % (i % 3)
        nd.compute_class()
    job = synth.job_c2(150)
    job.datacenters = ["dc0", "dc1", "dc2"]
    tg = job.task_groups[0]
    if kind == "even_and_targets":
        tg.spreads = [Spread("${node.datacenter}", 50, []),
                      Spread("${meta.rack}", 30, [SpreadTarget("r1", 20), SpreadTarget("r2", 30)])]
    elif kind == "per_node_values":
        tg.spreads = [Spread("${node.unique.name}", 40, [])]
    else:
        tg.affinities = [Affinity("${meta.rack}", "r1[0-9]", "regexp", 60)]
    eng, ora = _metrics_pair(nodes, allocs, job, synth.shuffle(len(nodes), 9))
    st = _view_metrics_protocol(eng, ora, 150)
    assert st["view"] >= 120, st


@pytest.mark.gpu
def test_metrics_view_rising_scores():
    """Scores that rise along the visit order (each node a little fuller than
    the one before): every option of a full pass enters the record's top-5
    heap for a moment, so k_trace_top's segment lists overflow and the
    record's heap is built by the sequential pass; the ScoreMetaData, order
    included, equal the oracle's."""
    from nomad_amd.structs import Affinity
    n = 3000
    nodes, allocs = [], []
    for i, nid in enumerate(sorted(synth.uuids(n, 21))):
        nd = synth.mock_node(nid)
        nd.name = "node-%05d" % i
        nd.compute_class()
        nodes.append(nd)
        allocs.append(Allocation(node_id=nid, job_id="fill", task_group="web", cpu_shares=1 + i,
                                 memory_mb=64, disk_mb=10, priority=50))
    job = synth.job_c2(24)
    job.task_groups[0].affinities = [Affinity("${node.class}", "no-such-class", "=", 50)]
    eng, ora = _metrics_pair(nodes, allocs, job, list(range(n)))
    st = _view_metrics_protocol(eng, ora, 24)
    assert st["view"] >= 16, st
