"""k_chain's instantiations (1, 4 and 16 visit positions per lane) on the same
lists, engine vs oracle ("k_chain shapes").

Round 3 dropped a one-position-per-lane k_chain that disagreed with the oracle
on a 500-node C5 list and faulted in the batch path. Its cause was a shape
constant, not the list: the wave-0 scan of the per-64-position tile counts
covered kChainTiles / 64 tiles per lane, which is 0 for a 1024-position
window (16 tiles), so no tile offset was ever computed and the option indices
built on them were wrong. The scan now derives its width from the shape
(ChainShape::kScanPer >= 1, static_asserts on every shape constant), the
kernel carries bounds guards (an option index past the window, more
re-evaluated rows than the redo list holds, a Select without a winner, a
record past the launch's count, more overlay rows than placements) that stop
the evaluation and fail the call with PE_EINTERNAL instead of storing out of
bounds, and every shape runs here against the oracle. PE_CHAIN_ITEMS asks for
a larger shape than the list needs; the engine never uses a smaller one.

Lists of at most 4096 positions with at most 256 placements run as one fused
launch (k_chain evaluates its first phase itself, carries the table build's
feasibility fold, builds the records and writes the placements back); the
"u" parameters run the same shapes unfused.
"""
import os

import numpy as np
import pytest

from nomad_amd import synth
from oracle.oracle import OracleGenericStack
from tests.helpers import assert_same_placements, run_place
from tests.test_chain_windows import big_job, one_slot_cluster

pytestmark = pytest.mark.gpu

# "1u" / "4u": the same shapes without the fused single launch (PE_CHAIN_FUSED
# set: k_base + k_chain + k_emit + k_emit_writeback as on longer lists)
SHAPES = ("1", "4", "16", "1u", "4u")


@pytest.fixture
def shape(request, monkeypatch):
    monkeypatch.setenv("PE_CHAIN_ITEMS", request.param.rstrip("u"))
    if request.param.endswith("u"):
        monkeypatch.setenv("PE_CHAIN_FUSED", "0")
    else:
        monkeypatch.delenv("PE_CHAIN_FUSED", raising=False)
    return request.param


def _engine(**kw):
    from nomad_amd.stack import GenericStack
    return GenericStack(**kw)


@pytest.mark.parametrize("shape", SHAPES, indirect=True)
def test_c5_500_node_list(shape):
    # the list the dropped variant disagreed on: device asks, windowed chain
    nodes, allocs = synth.cluster_c5(500, seed=1)
    job = synth.job_c5(120)
    perm = synth.shuffle(len(nodes), 11)
    _, lo, ro = run_place(OracleGenericStack, nodes, allocs, job, perm)
    _, le, re = run_place(_engine, nodes, allocs, job, perm)
    assert lo == le
    assert_same_placements(re, ro)
    assert [x.device_offers for x in re] == [x.device_offers for x in ro]


@pytest.mark.parametrize("shape", SHAPES, indirect=True)
@pytest.mark.parametrize("n,extra", [(900, 40), (1000, -7), (3000, -3)])
def test_fill_cluster(shape, n, extra):
    # Selects that walk the whole list, the full-window retry, the exhausted stream
    nodes = one_slot_cluster(n, seed=n + 1)
    job = big_job(n + extra)
    perm = synth.shuffle(n, 12)
    _, _, ro = run_place(OracleGenericStack, nodes, [], job, perm)
    _, _, re = run_place(_engine, nodes, [], job, perm)
    assert_same_placements(re, ro)


@pytest.mark.parametrize("shape", SHAPES, indirect=True)
def test_c1_dropin(shape):
    from tests.test_dropin import assert_equal_runs, both
    nodes, allocs = synth.cluster_c1(100, seed=42)
    job = synth.mock_job(count=10)
    a, b, _ = both(nodes, allocs, job, list(synth.shuffle(100, 3)), count=10)
    assert_equal_runs(a, b)


@pytest.mark.parametrize("shape", SHAPES, indirect=True)
def test_batch_path(shape):
    # the batch path: a persistent grid over many evaluations, row-indexed base
    from nomad_amd.stack import GenericStack
    nodes, allocs = synth.cluster_c5(500, seed=1)
    job = synth.job_c5(120)
    orders = np.stack([synth.shuffle(len(nodes), 100 + e) for e in range(24)])
    st = GenericStack()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.StageOrders(orders)
    rows, _, _, placed = st.PlaceBatch(0, 120)
    for e in (0, 7, 23):
        o = OracleGenericStack()
        o.SetState(nodes, allocs)
        o.SetJob(job)
        o.SetNodes(orders[e])
        ro = o.Place(0, 120)
        assert int(placed[e]) == len(ro)
        assert [int(r) for r in rows[e][:len(ro)]] == [x.row for x in ro]
