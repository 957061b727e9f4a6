"""GPU parity: the HIP engine against the oracle on identical seeded inputs.

Bar (BASELINE.json north_star): chosen node rows, cursor offsets and filter /
exhaust counts bit-exact; float64 scores bit-exact (same portable Pow
algorithm on both sides; the 1e-12 relative bound vs Go is the documented
tolerance, see oracle/gomath.h).
"""
import numpy as np
import pytest

from nomad_amd import synth
from nomad_amd.structs import Allocation, Constraint, SchedulerConfig
from oracle.oracle import OracleGenericStack, OracleSystemStack
from tests.helpers import assert_same_placements, run_place

pytestmark = pytest.mark.gpu


def engine_generic(**kw):
    from nomad_amd.stack import GenericStack
    return GenericStack(**kw)


def engine_system(**kw):
    from nomad_amd.stack import SystemStack
    return SystemStack(**kw)


def test_c1_mock_nodes_count10():
    nodes, allocs = synth.cluster_c1(100, seed=42)
    job = synth.mock_job(count=10)
    perm = synth.shuffle(len(nodes), 1)
    _, lim_o, ro = run_place(OracleGenericStack, nodes, allocs, job, perm)
    _, lim_e, re = run_place(engine_generic, nodes, allocs, job, perm)
    assert lim_o == lim_e == 7
    assert len(ro) == 10
    assert_same_placements(re, ro)


@pytest.mark.parametrize("n,count,seed", [(1000, 300, 3), (10000, 1000, 1), (64, 150, 5), (65, 150, 6),
                                          (130, 300, 7), (200, 700, 8)])
def test_c2_binpack_windowed(n, count, seed):
    nodes, allocs = synth.cluster_c2(n, seed=42)
    job = synth.job_c2(count)
    perm = synth.shuffle(len(nodes), seed)
    _, lo, ro = run_place(OracleGenericStack, nodes, allocs, job, perm)
    _, le, re = run_place(engine_generic, nodes, allocs, job, perm)
    assert lo == le
    assert_same_placements(re, ro)


def test_c2_spread_algorithm():
    nodes, allocs = synth.cluster_c2(2000, seed=5)
    job = synth.job_c2(400)
    perm = synth.shuffle(len(nodes), 9)
    cfg = SchedulerConfig(algorithm="spread")
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm, config=cfg)
    _, _, re = run_place(engine_generic, nodes, allocs, job, perm, config=cfg)
    assert_same_placements(re, ro)


def test_c3_spread_affinity_semver_regexp():
    nodes, allocs = synth.cluster_c3(3000, seed=7)
    job = synth.job_c3(300)
    perm = synth.shuffle(len(nodes), 2)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm)
    _, _, re = run_place(engine_generic, nodes, allocs, job, perm)
    assert_same_placements(re, ro)


def test_exhaustion_until_full():
    """Small cluster, large count: placements run until no node fits (nil option)."""
    nodes, allocs = synth.cluster_c2(50, seed=8)
    job = synth.job_c2(5000)
    perm = synth.shuffle(len(nodes), 4)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm)
    _, _, re = run_place(engine_generic, nodes, allocs, job, perm)
    assert ro[-1].row == -1
    assert_same_placements(re, ro)


def test_select_commit_path_matches_place():
    nodes, allocs = synth.cluster_c2(500, seed=3)
    job = synth.job_c2(50)
    perm = synth.shuffle(len(nodes), 6)
    o = OracleGenericStack(); o.SetState(nodes, allocs); o.SetJob(job); o.SetNodes(list(perm))
    e = engine_generic(); e.SetState(nodes, allocs); e.SetJob(job); e.SetNodes(list(perm))
    for _ in range(50):
        a, b = o.SelectRaw(0), e.SelectRaw(0)
        assert_same_placements([b], [a])
        if a.row < 0:
            break
        o.Commit(0, a.row)
        e.Commit(0, b.row)


def test_sweep_select_path_matches_oracle(monkeypatch):
    """Full-scan Selects through the multi-CU sweep + SweepRec reduction (forced
    with PE_SWEEP_MIN=1) against the oracle, Select -> Commit for 80 placements."""
    monkeypatch.setenv("PE_SWEEP_MIN", "1")
    nodes, allocs = synth.cluster_c3(2500, seed=13)
    job = synth.job_c3(80)
    perm = synth.shuffle(len(nodes), 8)
    o = OracleGenericStack(); o.SetState(nodes, allocs); o.SetJob(job); o.SetNodes(list(perm))
    e = engine_generic(); e.SetState(nodes, allocs); e.SetJob(job); e.SetNodes(list(perm))
    for _ in range(80):
        a, b = o.SelectRaw(0), e.SelectRaw(0)
        assert_same_placements([b], [a])
        if a.row < 0:
            break
        o.Commit(0, a.row)
        e.Commit(0, b.row)


def test_sweep_select_nonpositive_demotion(monkeypatch):
    """All options score <= 0 (anti-affinity dominates): the first three
    non-positive options are demoted behind the rest (select.go:35-74)."""
    monkeypatch.setenv("PE_SWEEP_MIN", "1")
    nodes, _ = synth.cluster_c3(300, seed=2)
    job = synth.job_c3(2)          # desired count 2: each collision costs -(c+1)/2
    allocs = [Allocation(node_id=n.id, job_id=job.id, task_group="web") for n in nodes for _ in range(3)]
    perm = synth.shuffle(len(nodes), 4)
    for use_sweep in ("1", "1000000"):
        monkeypatch.setenv("PE_SWEEP_MIN", use_sweep)
        o = OracleGenericStack(); o.SetState(nodes, allocs); o.SetJob(job); o.SetNodes(list(perm))
        e = engine_generic(); e.SetState(nodes, allocs); e.SetJob(job); e.SetNodes(list(perm))
        a, b = o.SelectRaw(0), e.SelectRaw(0)
        assert a.row >= 0 and a.final_score <= 0
        assert_same_placements([b], [a])


@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_batch_evals_match_single_eval_oracle(cfg):
    """pe_place_batch: every concurrent eval equals SetNodes(order) + Place on the oracle."""
    if cfg == "c2":
        nodes, allocs = synth.cluster_c2(2000, seed=21)
        job = synth.job_c2(300)
    else:
        nodes, allocs = synth.cluster_c3(1500, seed=4)
        job = synth.job_c3(120)
    E = 6
    orders = np.stack([synth.shuffle(len(nodes), 100 + e) for e in range(E)])
    e = engine_generic()
    e.SetState(nodes, allocs)
    e.SetJob(job)
    e.StageOrders(orders)
    count = job.task_groups[0].count
    rows, scores, evaluated, placed = e.PlaceBatch(0, count)
    for k in range(E):
        _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, orders[k])
        assert placed[k] == sum(1 for r in ro if r.row >= 0)
        for i, r in enumerate(ro):
            assert rows[k, i] == r.row, (k, i)
            assert evaluated[k, i] == r.nodes_evaluated, (k, i)
            if r.row >= 0:
                assert scores[k, i] == r.final_score, (k, i)


def test_batch_result_paths_agree(monkeypatch):
    """Windowed batch records streamed into mapped host memory (64-record LDS
    flushes, ragged tail, early nil stop) equal the device-buffer + copy path
    and the oracle."""
    nodes, allocs = synth.cluster_c2(12, seed=12)
    job = synth.job_c2(1000)          # exhausts the cluster mid-way: nil option ends each eval
    E = 5
    orders = np.stack([synth.shuffle(len(nodes), 300 + e) for e in range(E)])
    res = []
    for via_copy in ("0", "1"):
        monkeypatch.setenv("PE_RESULTS_VIA_COPY", via_copy)
        e = engine_generic()
        e.SetState(nodes, allocs)
        e.SetJob(job)
        e.StageOrders(orders)
        res.append(e.PlaceBatch(0, 1000))
        e.close()
    assert np.array_equal(res[0][3], res[1][3])
    for k in range(E):   # records past the nil stop are undefined
        m = min(int(res[0][3][k]) + 1, 1000)
        for a, b in zip(res[0][:3], res[1][:3]):
            assert np.array_equal(a[k, :m], b[k, :m])
    rows, scores, evaluated, placed = res[0]
    for k in range(E):
        _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, orders[k])
        got = int(placed[k])
        assert got == sum(1 for r in ro if r.row >= 0) and 0 < got < 1000
        for i, r in enumerate(ro):
            assert rows[k, i] == r.row and evaluated[k, i] == r.nodes_evaluated, (k, i)
            if r.row >= 0:
                assert scores[k, i] == r.final_score, (k, i)


@pytest.mark.parametrize("n,count", [(40, 400), (3000, 900), (10000, 1000)])
def test_phase_loop_matches_lazy_loop(monkeypatch, n, count):
    """The phase-static windowed loop (k_base + k_chain: one rotation of the
    visit list resolved at a time) equals the lazy per-position loop (k_window)
    and the oracle, batched and single-eval, including walks that wrap the
    list many times and an exhausted stream; a visit list with repeated rows
    takes the lazy loop."""
    nodes, allocs = synth.cluster_c2(n, seed=31)
    job = synth.job_c2(count)
    rng = np.random.Generator(np.random.PCG64(77))
    orders = np.stack([synth.shuffle(n, 500 + e) for e in range(3)])
    dup = synth.shuffle(n, 600).copy()
    dup[rng.integers(0, n, size=n // 4)] = dup[rng.integers(0, n, size=n // 4)]   # repeated rows
    res = []
    for lazy in ("1", "0"):
        monkeypatch.setenv("PE_WINDOW_LAZY", lazy)
        e = engine_generic()
        e.SetState(nodes, allocs)
        e.SetJob(job)
        e.StageOrders(orders)
        res.append(e.PlaceBatch(0, count))
        single = []
        for order in list(orders) + [dup]:
            e.ResetPlan()
            e.SetJob(job)
            e.SetNodes(order)
            single.append(e.Place(0, count))
        res.append(single)
        e.close()
    (b_lazy, s_lazy, b_chain, s_chain) = res
    assert np.array_equal(b_lazy[3], b_chain[3])
    for k in range(len(orders)):
        m = min(int(b_chain[3][k]) + 1, count)
        for a, b in zip(b_lazy[:3], b_chain[:3]):
            assert np.array_equal(a[k, :m], b[k, :m]), k
    for k, order in enumerate(list(orders) + [dup]):
        assert_same_placements(s_chain[k], s_lazy[k])
        _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, order)
        assert_same_placements(s_chain[k], ro)


@pytest.mark.parametrize("kind", ["c3", "c4"])
def test_columnar_cluster_place(kind):
    """Vectorised (columnar) snapshot path: full count loop vs the oracle on the same tables."""
    from nomad_amd import synth_columnar
    cs = synth_columnar.ColumnarState(20000, seed=5, kind=kind, prefill=0.05)
    job = synth.job_c3(200) if kind == "c3" else synth.job_c2(200)
    perm = np.random.Generator(np.random.PCG64(9)).permutation(20000).astype(np.uint32)
    res = []
    for cls in (OracleGenericStack, engine_generic):
        st = cls()
        st.SetStateColumnar(cs)
        st.SetJob(job)
        st.SetNodes(perm)
        res.append(st.Place(0, 200))
    assert_same_placements(res[1], res[0])


def test_system_job_sweep():
    nodes, allocs = synth.cluster_c4(3000, seed=11)
    job = synth.mock_system_job()
    perm = synth.shuffle(len(nodes), 5)
    res = []
    for cls in (OracleSystemStack, engine_system):
        st = cls()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(list(perm))
        res.append(st.SystemPlace(0))
    (so, to, po), (se, te, pe) = res
    assert po == pe
    assert np.array_equal(to, te)
    placed = to == 0
    assert np.array_equal(so[placed], se[placed])
