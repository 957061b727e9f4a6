"""Parity at the BASELINE.json configs' own sizes (VERDICT r1 "configs untested").

C4: the system job on the 100k-node cluster, engine vs oracle unsharded, and
the per-rank contiguous ranges of the SetNodes list (nomad_amd/shard.py) for
N = 2, 4, 8 run one after another in this process: their union must equal the
unsharded placement (scheduler_system.go:283-425; each node's Select is
independent).

C5: device asks with service preemption on 50k nodes, a cluster whose GPU nodes
are all but a handful fully held by priority-20 work, so most placements evict
(preemption.go:198-557), through the fused count loop and through the caller's
Select / Commit protocol; engine vs oracle placement by placement, preempted
sets included.

C2 at 10k nodes and the 1000-placement count: the caller protocol vs the oracle.
"""
import numpy as np
import pytest

from nomad_amd import shard, synth, synth_columnar
from nomad_amd.structs import SchedulerConfig
from oracle.oracle import OracleGenericStack, OracleSystemStack
from tests.helpers import assert_same_placements

pytestmark = pytest.mark.gpu


def test_c4_100k_system_job_and_range_shards():
    from nomad_amd.stack import SystemStack
    n = 100000
    cs = synth_columnar.ColumnarState(n, seed=11, kind="c4", prefill=0.05)
    job = synth.mock_system_job()
    rows = np.random.Generator(np.random.PCG64(5)).permutation(n).astype(np.uint32)
    o = OracleSystemStack()
    o.SetStateColumnar(cs)
    o.SetJob(job)
    o.SetNodes(rows)
    so, to, po = o.SystemPlace(0)
    e = SystemStack()
    e.SetStateColumnar(cs)
    e.SetJob(job)
    e.SetNodes(rows)
    se, te, pe = e.SystemPlace(0)
    assert pe == po and np.array_equal(te, to)
    placed = to == 0
    assert np.array_equal(se[placed], so[placed])
    assert 0.5 * n < po < n           # ~10 % filtered (windows), ~5 % exhausted (pre-filled)
    assert (to == 1).sum() > 0.05 * n and (to == 2).sum() > 0.01 * n
    for world in (2, 4, 8):
        score = np.empty(n)
        status = np.empty(n, dtype=np.uint8)
        total = 0
        for rank in range(world):
            e.ResetPlan()
            e.SetJob(job)
            b, end, sc, st, p = shard.system_place_sharded(e, rows, rank, world)
            score[b:end], status[b:end] = sc, st
            total += p
        assert total == po, world
        assert np.array_equal(status, to), world
        assert np.array_equal(score[placed], so[placed]), world


@pytest.fixture(scope="module")
def c5_cluster():
    return synth.cluster_c5(50000, seed=5, busy=0.9995)


def test_c5_50k_preemption_count_loop(c5_cluster):
    from nomad_amd.stack import GenericStack
    nodes, allocs = c5_cluster
    job = synth.job_c5(70)
    perm = synth.shuffle(len(nodes), 77)
    cfg = SchedulerConfig(preempt_service=True)
    res = []
    for cls in (OracleGenericStack, GenericStack):
        st = cls(config=cfg)
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
        res.append(st.Place(0, 70))
    ro, re = res
    assert_same_placements(re, ro)
    assert [sorted(x.preempted) for x in re] == [sorted(x.preempted) for x in ro]
    assert [x.device_offers for x in re] == [x.device_offers for x in ro]
    evicting = sum(1 for x in ro if x.preempted)
    assert len(ro) == 70 and evicting >= 40, evicting


def test_c5_50k_caller_protocol(c5_cluster):
    from nomad_amd.stack import GenericStack
    from tests.test_dropin import compute_placements
    nodes, allocs = c5_cluster
    job = synth.job_c5(60)
    perm = synth.shuffle(len(nodes), 78)
    cfg = SchedulerConfig(preempt_service=True)
    res = []
    for cls in (OracleGenericStack, GenericStack):
        st = cls(config=cfg)
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
        res.append(compute_placements(st, 60, preempt=True))
    assert res[0] == res[1]
    assert sum(1 for x in res[0] if x is not None and x[7]) >= 30


@pytest.fixture(scope="module")
def c5_bench_shape():
    """bench.py's C5 workload exactly (section_c5): 50k nodes, busy=0.99,
    job_c5(1000), shuffle(.., 77), service preemption on, and the oracle's
    1000 placements of it frozen in tests/golden/c5_bench_shape.json.gz
    (tools/make_c5_golden.py: ~10 minutes of oracle time, too long for a GPU
    test; tests/test_golden.py re-derives its first placements on the CPU).
    The oracle's Place is the caller's loop itself (oracle.cpp oracle_place:
    Select, Preempt retry on nil as generic_sched.go:773-792, commit with the
    preempted set), so the one fixture answers both engine protocols below."""
    from tools.make_c5_golden import OUT, build
    import gzip
    import json
    with gzip.open(OUT, "rt") as f:
        g = json.load(f)
    nodes, allocs, job, perm, cfg = build(g["case"])
    return nodes, allocs, job, perm, cfg, g


def _c5_key(r):
    # the record fields the fixture holds, as tests/test_dropin._key orders them
    return (r.row, r.final_score.hex(), tuple(s.hex() for s in r.scores), r.nodes_evaluated, r.nodes_filtered,
            r.nodes_exhausted, r.new_offset, tuple(r.preempted), tuple(r.device_offers))


def _c5_want(g):
    return [(w["row"], w["final_score"], tuple(w["scores"]), w["evaluated"], w["filtered"], w["exhausted"],
             w["offset"], tuple(w["preempted"]), tuple(w["device_offers"])) for w in g["placements"]]


def test_c5_bench_shape_count_loop(c5_bench_shape):
    # the engine's device count loop (k_ploop) over all 1000 placements
    from nomad_amd.stack import GenericStack
    nodes, allocs, job, perm, cfg, g = c5_bench_shape
    st = GenericStack(config=cfg)
    st.SetState(nodes, allocs)
    st.SetJob(job)
    assert st.SetNodes(perm) == g["limit"]
    got = [_c5_key(r) for r in st.Place(0, 1000)]
    want = _c5_want(g)
    assert len(got) == len(want) == 1000
    for i, (x, y) in enumerate(zip(got, want)):
        assert x == y, ("placement %d" % i, x, y)
    assert sum(1 for w in want if w[7]) == 628


def test_c5_bench_shape_caller_protocol(c5_bench_shape):
    # the same evaluation through Select / Commit with the Preempt retry, every
    # Select through C: plain nils and Preempt options both from the run records
    from nomad_amd.stack import GenericStack, SelectOptions
    nodes, allocs, job, perm, cfg, g = c5_bench_shape
    st = GenericStack(config=cfg)
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes(perm)
    want = _c5_want(g)
    nils = {n[0]: tuple(n[1:]) for n in g["plain_nils"]}
    for i, w in enumerate(want):
        r = st.SelectRaw(0)
        if r.row < 0:
            assert (r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted, r.new_offset) == nils[i], i
            r = st.SelectRaw(0, SelectOptions(preempt=True))
        else:
            assert i not in nils, i
        assert r.row >= 0, "placement %d: nil" % i
        got = _c5_key(r)
        assert got == w, ("placement %d" % i, got, w)
        st.Commit(0, r.row, r.preempted)
    runs, served, rollbacks, records = st.SpeculationStats()
    # speculative runs of x4 growing length serve everything; no per-Select path
    assert rollbacks == 0 and runs <= 6 and served == len(want) + len(nils) - runs, st.SpeculationStats()


def test_c5_bench_shape_served_from_the_view(c5_bench_shape):
    # the Go shim's zero-crossing path: every answer it can take from the
    # served-Select view, the nils and PreemptedAllocs included
    from nomad_amd.stack import GenericStack
    from tests.test_spec_view import ViewAnswers, protocol_answers
    nodes, allocs, job, perm, cfg, g = c5_bench_shape
    st = GenericStack(config=cfg)
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes(perm)
    vc = ViewAnswers(st)
    got = [x if x[0] == "nil" else (x[0], x[1].hex(), tuple(v.hex() for v in x[2])) + tuple(x[3:])
           for x in protocol_answers(vc, 1000)]
    want, nils = _c5_want(g), {n[0]: n[1:] for n in g["plain_nils"]}
    exp = []
    for i, w in enumerate(want):
        if i in nils:
            exp.append(("nil",) + tuple(nils[i]))
        exp.append(w)
    assert len(got) == len(exp)
    for i, (x, y) in enumerate(zip(got, exp)):
        assert x == y, ("answer %d" % i, x, y)
    runs, _, rollbacks, _ = st.SpeculationStats()
    assert rollbacks == 0 and runs <= 6 and vc.served >= len(exp) - runs, (st.SpeculationStats(), vc.served)


def test_c2_10k_caller_protocol_count_1000():
    from nomad_amd.stack import GenericStack
    from tests.test_dropin import compute_placements
    nodes, allocs = synth.cluster_c2(10000, seed=42)
    job = synth.job_c2(1000)
    perm = synth.shuffle(len(nodes), 1001)
    res = []
    for cls in (OracleGenericStack, GenericStack):
        st = cls()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
        res.append(compute_placements(st, 1000))
    assert len(res[0]) == 1000 and res[0] == res[1]


@pytest.mark.gpu
def test_c2_100k_nodes_count_1000():
    # the metric's 100k-node case (BASELINE.json: "count=1000 job on 10k/100k
    # nodes"), limit 17 (stack.go:83-90): the phase-static chain over windows
    # of the long list, speculative behind Select / Commit
    import numpy as np
    from nomad_amd.stack import GenericStack
    from oracle.oracle import OracleGenericStack
    nodes, allocs = synth.cluster_c2(100000, seed=42)
    job = synth.job_c2(1000)
    perm = synth.shuffle(100000, 77)
    got = []
    for st in (GenericStack(), OracleGenericStack()):
        st.SetState(nodes, allocs)
        st.SetJob(job)
        assert st.SetNodes(perm) == 17
        seq = []
        for _ in range(1000):
            r = st.Select(0)
            seq.append(None if r is None else (r.row, r.final_score, r.nodes_evaluated, r.new_offset))
            if r is None:
                break
            st.Commit(0, r.row)
        got.append(seq)
    assert got[0] == got[1]


@pytest.mark.gpu
def test_chain_window_stall_on_sparse_long_list():
    # 40k nodes of which only a few hundred fit: a Select walks more than the
    # chain's 16384-position window, so the launch hands over to the lazy loop
    import numpy as np
    from nomad_amd.stack import GenericStack
    from oracle.oracle import OracleGenericStack
    from nomad_amd.structs import Allocation
    nodes, allocs = synth.cluster_c2(40000, seed=5, other_allocs=False)
    for i, nd in enumerate(nodes):
        if i % 150:
            allocs.append(Allocation(node_id=nd.id, job_id="filler", task_group="tg",
                                     cpu_shares=nd.cpu_shares - 100 - 200, memory_mb=64, disk_mb=10))
    job = synth.job_c2(400)
    perm = synth.shuffle(40000, 78)
    got = []
    for st in (GenericStack(), OracleGenericStack()):
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
        got.append([(r.row, r.final_score, r.nodes_evaluated, r.new_offset) for r in st.Place(0, 400)])
    assert got[0] == got[1]
