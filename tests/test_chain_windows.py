"""k_chain phase windows on clusters that fill up.

Every node takes exactly one placement of the job, so each later Select walks
past more exhausted nodes (feasible.go:90-117 keeps pulling until the
LimitIterator has `limit` options, select.go:35-74). Phases after the first
cover a window sized from the positions the earlier Selects consumed; here
that estimate falls short more and more, down to Selects that need the whole
list (the full-window retry and the exhausted stream). Engine vs oracle,
placement by placement, including the final nil Select when the count exceeds
the cluster.
"""
import numpy as np
import pytest

from nomad_amd import synth
from nomad_amd.structs import Job, NetworkResource, Task, TaskGroup
from oracle.oracle import OracleGenericStack
from tests.helpers import assert_same_placements, run_place

pytestmark = pytest.mark.gpu


def _engine(**kw):
    from nomad_amd.stack import GenericStack
    return GenericStack(**kw)


def one_slot_cluster(n, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = []
    for k, nid in enumerate(sorted(synth.uuids(n, seed))):
        nd = synth.mock_node(nid)
        nd.name = "node-%05d" % k
        nd.cpu_shares = int(rng.integers(4000, 6000))   # one 3000 MHz ask fits, two do not
        nd.memory_mb = int(rng.choice([8192, 16384]))
        nd.compute_class()
        nodes.append(nd)
    return nodes


def big_job(count):
    return Job(id="fill", task_groups=[TaskGroup(
        name="web", count=count, ephemeral_disk_mb=150,
        network=NetworkResource(mode="host", dynamic_ports=1, host_network="default"),
        tasks=[Task(name="web", driver="exec", cpu=3000, memory_mb=256)])])


@pytest.mark.parametrize("n,extra", [(3000, -3), (2500, 40), (9000, -200)])
def test_chain_fills_cluster(n, extra):
    nodes = one_slot_cluster(n, seed=n)
    job = big_job(n + extra)
    perm = synth.shuffle(n, 11)
    _, _, ro = run_place(OracleGenericStack, nodes, [], job, perm)
    _, _, re = run_place(_engine, nodes, [], job, perm)
    assert_same_placements(re, ro)
    placed = sum(1 for x in re if x.row >= 0)
    assert placed == min(n, n + extra)
    if extra > 0:
        assert re[-1].row < 0


def test_dropin_chain_stall_on_sparse_options():
    """The caller's Select/Commit protocol on a list longer than one chain
    window whose options thin out: the speculative run starts on the chain
    (compact records) and hands over to the lazy loop when a Select no longer
    stops inside the window; every Select must still equal the oracle's."""
    from nomad_amd.structs import Constraint
    from tests.test_dropin import assert_equal_runs, both
    n = 20000
    nodes = one_slot_cluster(n, seed=77)
    for k, nd in enumerate(nodes):
        nd.datacenter = "dc1" if (k < 200 or k % 997 == 0) else "dc2"
        nd.compute_class()
    job = big_job(260)
    job.constraints = [Constraint("${node.datacenter}", "dc1", "=")]
    a, b, eng = both(nodes, [], job, list(range(n)), count=260)
    assert_equal_runs(a, b)
    assert a[-1] is None and sum(1 for x in a if x is not None) == 220
