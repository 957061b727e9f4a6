"""Multi-process sharding on CPU ranks over gloo, world size 2.

The product path runs one process per GPU over RCCL; here the same driver code
(nomad_amd/shard.py) runs on CPU processes with the oracle standing in for the
per-shard device work (the oracle is test infrastructure): system placements
over contiguous list ranges, and full-pass Selects whose 80-byte records are
all-gathered and merged every placement. Both must equal one process running
the whole evaluation. The GPU test checks the engine's own shard records.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from nomad_amd import shard, synth
from nomad_amd.structs import SchedulerConfig


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _system_worker(rank, world, port, q):
    from oracle.oracle import OracleSystemStack
    _init(rank, world, port)
    nodes, allocs = synth.cluster_c4(1200, seed=11)
    job = synth.mock_system_job()
    rows = synth.shuffle(len(nodes), 3)
    st = OracleSystemStack()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    b, e, score, status, placed = shard.system_place_sharded(st, rows, rank, world)
    got = [None] * world
    dist.all_gather_object(got, (b, e, score.tolist(), status.tolist(), placed))
    if rank == 0:
        q.put(got)
    dist.destroy_process_group()


def _fullscan_worker(rank, world, port, q):
    from oracle.shard_rec import OracleShardStack
    _init(rank, world, port)
    nodes, allocs = synth.cluster_c3(900, seed=21)
    job = synth.job_c3(60)
    perm = synth.shuffle(len(nodes), 4)
    st = OracleShardStack()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes(list(perm))
    sf = shard.ShardedFullScan(st, len(nodes), dist)
    res = sf.Place(0, 60)
    if rank == 0:
        q.put([(r.row, r.final_score, r.nodes_filtered, r.nodes_exhausted) for r in res])
    dist.destroy_process_group()


def _run(worker, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return out


def test_shard_range_partitions():
    for n in (0, 1, 7, 100000):
        for w in (1, 2, 3, 8):
            spans = [shard.shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_system_sharded_gloo_matches_single_process():
    from oracle.oracle import OracleSystemStack
    got = _run(_system_worker)
    nodes, allocs = synth.cluster_c4(1200, seed=11)
    job = synth.mock_system_job()
    rows = synth.shuffle(len(nodes), 3)
    st = OracleSystemStack()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes(list(rows))
    score, status, placed = st.SystemPlace(0)
    cat_status = np.concatenate([np.asarray(g[3], dtype=np.uint8) for g in got])
    cat_score = np.concatenate([np.asarray(g[2]) for g in got])
    assert sum(g[4] for g in got) == placed
    assert np.array_equal(cat_status, status)
    m = status == 0
    assert np.array_equal(cat_score[m], score[m])


def test_full_scan_sharded_gloo_matches_single_process():
    from oracle.oracle import OracleGenericStack
    got = _run(_fullscan_worker)
    nodes, allocs = synth.cluster_c3(900, seed=21)
    job = synth.job_c3(60)
    perm = synth.shuffle(len(nodes), 4)
    st = OracleGenericStack()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes(list(perm))
    ref = st.Place(0, 60)
    assert [(r.row, r.final_score, r.nodes_filtered, r.nodes_exhausted) for r in ref] == [tuple(x) for x in got]


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [1, 2, 3, 8])
def test_engine_shard_records_match_select(shards):
    """pe_select_shard over disjoint row ranges + pe_select_merge == pe_select,
    placement after placement (single process, shards as row ranges)."""
    from nomad_amd.stack import GenericStack
    nodes, allocs = synth.cluster_c3(5000, seed=22)
    job = synth.job_c3(40)
    perm = synth.shuffle(len(nodes), 8)
    a, b = GenericStack(), GenericStack()
    for st in (a, b):
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(list(perm))
    for _ in range(40):
        recs = [a.SelectShard(0, *shard.shard_range(len(nodes), r, shards)) for r in range(shards)]
        x = a.SelectMerge(0, recs)
        y = b.SelectRaw(0)
        assert (x.row, x.final_score, x.scores, x.nodes_filtered, x.nodes_exhausted, x.new_offset) == \
               (y.row, y.final_score, y.scores, y.nodes_filtered, y.nodes_exhausted, y.new_offset)
        if x.row < 0:
            break
        a.Commit(0, x.row)
        b.Commit(0, y.row)


def _plan_worker(rank, world, port, q):
    from nomad_amd.plan import assemble_result
    from nomad_amd.synth_plan import random_case
    from oracle import plan_apply as O
    _init(rank, world, port)
    nodes, allocs, plan = random_case(31, n_nodes=40)
    my_nodes, my_allocs, my_plan = shard.shard_plan(nodes, allocs, plan, rank, world)
    snap = O.Snapshot(my_nodes, my_allocs)
    ids, fits, why = O.evaluate_plan_placements(snap, my_plan)
    got = [None] * world
    dist.all_gather_object(got, list(zip(ids, fits, why)))
    if rank == 0:
        q.put(got)
    dist.destroy_process_group()


def test_plan_apply_sharded_equals_single():
    """Plan applier over 2 gloo ranks (contiguous node ranges, no collective on
    the data path) gives the same per-node outcomes as one process."""
    from oracle import plan_apply as O
    from nomad_amd.synth_plan import random_case
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_plan_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    merged = {nid: (fit, why) for part in got for nid, fit, why in part}
    nodes, allocs, plan = random_case(31, n_nodes=40)
    ids, fits, why = O.evaluate_plan_placements(O.Snapshot(nodes, allocs), plan)
    assert merged == {nid: (f, w) for nid, f, w in zip(ids, fits, why)}
    assert sum(len(part) for part in got) == len(ids)


@pytest.mark.gpu
@pytest.mark.parametrize("n,count", [(5000, 300), (20000, 120)])
def test_engine_rccl_sharded_loop_matches_place(n, count):
    """pe_place_sharded (RCCL all-gather of the records on the engine stream
    between k_sweep and k_sweep_step) at one rank == pe_place's device loop ==
    the oracle, record by record."""
    from nomad_amd.stack import GenericStack
    from oracle.oracle import OracleGenericStack
    nodes, allocs = synth.cluster_c3(n, seed=23)
    job = synth.job_c3(count)
    perm = synth.shuffle(len(nodes), 9)
    a, b = GenericStack(), GenericStack()
    for st in (a, b):
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(list(perm))
    rank, world = shard.comm_init(a)
    assert (rank, world) == (0, 1)
    got = shard.device_place(a, 0, count, len(nodes), rank, world)
    ref = b.Place(0, count)

    def key(r):
        return (r.row, r.final_score, tuple(r.scores), r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted)
    assert [key(r) for r in got] == [key(r) for r in ref]
    if n <= 5000:
        o = OracleGenericStack()
        o.SetState(nodes, allocs)
        o.SetJob(job)
        o.SetNodes(list(perm))
        assert [(r.row, r.final_score) for r in got] == [(r.row, r.final_score) for r in o.Place(0, count)]
    # the plan is shared: the next Select on both handles agrees
    x, y = a.SelectRaw(0), b.SelectRaw(0)
    assert (x.row, x.final_score) == (y.row, y.final_score)


def _engine_system_worker(rank, world, port, q):
    # one engine process per rank, every rank on the box's GPU 0 at the same
    # time (the one-GPU rehearsal of the per-GPU processes): its contiguous
    # range of the SetNodes list, no data-path collective
    from nomad_amd import synth_columnar
    from nomad_amd.stack import SystemStack
    _init(rank, world, port)
    n = 100000
    cs = synth_columnar.ColumnarState(n, seed=11, kind="c4", prefill=0.05)
    job = synth.mock_system_job()
    rows = np.random.Generator(np.random.PCG64(5)).permutation(n).astype(np.uint32)
    st = SystemStack(device=0)
    st.SetStateColumnar(cs)
    st.SetJob(job)
    dist.barrier()   # the ranks' placements run concurrently
    b, e, score, status, placed = shard.system_place_sharded(st, rows, rank, world)
    got = [None] * world
    dist.all_gather_object(got, (b, e, score.tolist(), status.tolist(), placed))
    st.close()
    if rank == 0:
        q.put(got)
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_c4_concurrent_rank_processes_match_oracle(world):
    """C4 at its full 100k nodes, `world` engine processes placing their
    shards concurrently on one GPU: the union equals the oracle's unsharded
    placement (tests/test_full_size.py runs the same shards one after another)."""
    from nomad_amd import synth_columnar
    from oracle.oracle import OracleSystemStack
    got = _run(_engine_system_worker, world)
    n = 100000
    cs = synth_columnar.ColumnarState(n, seed=11, kind="c4", prefill=0.05)
    job = synth.mock_system_job()
    rows = np.random.Generator(np.random.PCG64(5)).permutation(n).astype(np.uint32)
    o = OracleSystemStack()
    o.SetStateColumnar(cs)
    o.SetJob(job)
    o.SetNodes(rows)
    so, to, po = o.SystemPlace(0)
    score = np.empty(n)
    status = np.empty(n, dtype=np.uint8)
    total = 0
    for b, e, sc, st, p in got:
        score[b:e], status[b:e] = sc, st
        total += p
    assert total == po and np.array_equal(status, to)
    placed = to == 0
    assert np.array_equal(score[placed], so[placed])


def _engine_fullscan_worker(rank, world, port, q):
    # one engine per rank, every rank on the box's GPU 0, the per-placement
    # record exchange over gloo (pe_comm_init_host): the sharded count loop of
    # pe_place_sharded with two ranks, engine on both sides
    from nomad_amd.stack import GenericStack
    _init(rank, world, port)
    n, count = 6000, 150
    nodes, allocs = synth.cluster_c3(n, seed=24)
    job = synth.job_c3(count)
    perm = synth.shuffle(n, 10)
    st = GenericStack(device=0)
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes(list(perm))
    shard.host_comm_init(st, dist)
    got = shard.device_place(st, 0, count, n, rank, world)
    stats = st.last_exchange_stats()
    nxt = st.SelectRaw(0)   # the plan is the same on every rank afterwards
    st.close()
    keys = [(r.row, r.final_score, tuple(r.scores), r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted)
            for r in got]
    allk = [None] * world
    dist.all_gather_object(allk, (keys, (nxt.row, nxt.final_score), stats))
    if rank == 0:
        q.put(allk)
    dist.destroy_process_group()


@pytest.mark.gpu
def test_engine_sharded_loop_two_ranks_over_gloo():
    """pe_place_sharded at world size 2: two engine processes on one GPU, each
    sweeping half the rows into one merged record per placement, the records
    all-gathered through torch.distributed (gloo) by the engine's host
    transport. Both ranks return pe_place's records and the oracle's rows."""
    from nomad_amd.stack import GenericStack
    from oracle.oracle import OracleGenericStack
    got = _run(_engine_fullscan_worker, 2)
    n, count = 6000, 150
    nodes, allocs = synth.cluster_c3(n, seed=24)
    job = synth.job_c3(count)
    perm = synth.shuffle(n, 10)
    b, o = GenericStack(), OracleGenericStack()
    for st in (b, o):
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(list(perm))
    ref = b.Place(0, count)
    keys = [(r.row, r.final_score, tuple(r.scores), r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted)
            for r in ref]
    oref = [(r.row, r.final_score) for r in o.Place(0, count)]
    nb, no = b.SelectRaw(0), o.SelectRaw(0)
    for k, nxt, stats in got:
        assert k == keys
        assert [(x[0], x[1]) for x in k] == oref
        assert nxt == (nb.row, nb.final_score) == (no.row, no.final_score)
        assert stats[3] == count   # every placement exchanged once
