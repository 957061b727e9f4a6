"""Property sets past the LDS tables: spread and
distinct_property sets of any number of values and up to 16 sets per task
group. propertySet (scheduler/propertyset.go:14-355) keeps an unbounded map
of value -> count; SpreadIterator (spread.go:96-228) scores against it. The
engine lays the per-value tables out set after set and keeps them in LDS while
they fit, in HBM beyond; the even-spread min / max is a block reduction over
any number of values. Engine vs oracle, placement by placement.
"""
import numpy as np
import pytest

from nomad_amd import synth
from nomad_amd.structs import Constraint, Job, Spread, SpreadTarget, Task, TaskGroup
from oracle.oracle import OracleGenericStack
from tests.helpers import assert_same_placements, run_place

pytestmark = pytest.mark.gpu


def _engine(**kw):
    from nomad_amd.stack import GenericStack
    return GenericStack(**kw)


def cluster(n, seed, slots=0, zones=0):
    """The C3 cluster with escaped high-cardinality properties: meta
    unique.slot (`slots` values) and unique.zone (`zones` values), neither in
    the computed class."""
    nodes, allocs = synth.cluster_c3(n, seed=seed)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    for k, nd in enumerate(nodes):
        if slots:
            nd.meta["unique.slot"] = "s%05d" % (k % slots)
        if zones:
            nd.meta["unique.zone"] = "z%04d" % int(rng.integers(0, zones))
        nd.compute_class()
    return nodes, allocs


def job(count, spreads=(), constraints=(), tg_constraints=()):
    return Job(id="wide-ps", priority=50, datacenters=["dc1", "dc2", "dc3"],
               constraints=[Constraint("${attr.kernel.name}", "linux", "=")] + list(constraints),
               spreads=list(spreads),
               task_groups=[TaskGroup(name="web", count=count, ephemeral_disk_mb=150,
                                      constraints=list(tg_constraints),
                                      tasks=[Task(name="web", driver="exec", cpu=250, memory_mb=128)])])


def _both(nodes, allocs, jb, perm):
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, jb, perm)
    _, _, re = run_place(_engine, nodes, allocs, jb, perm)
    assert_same_placements(re, ro)
    return re


def test_even_spread_over_every_node_lds_tables():
    # ${node.unique.name}: one value per node (3000), tables ~37 KB in LDS
    nodes, allocs = cluster(3000, seed=3)
    jb = job(60, spreads=[Spread("${node.unique.name}", 50)],
             constraints=[Constraint("${meta.rack}", "3", "distinct_property")])
    re = _both(nodes, allocs, jb, synth.shuffle(len(nodes), 1))
    assert sum(1 for x in re if x.row >= 0) == 60


def test_spread_tables_in_hbm():
    # 6000 values: the tables pass the LDS budget and live in HBM
    nodes, allocs = cluster(6000, seed=5, slots=6000)
    targets = [SpreadTarget("s%05d" % k, 1) for k in range(0, 6000, 97)]
    jb = job(120, spreads=[Spread("${meta.unique.slot}", 70, targets), Spread("${node.datacenter}", 30,
                                                                              [SpreadTarget("dc1", 60)])])
    _both(nodes, allocs, jb, synth.shuffle(len(nodes), 2))


def test_targets_over_many_values_and_six_sets():
    """Three spreads (one with 40 one-percent targets over 700 values) and three
    distinct_property sets: 6 sets, more than round 3's 4."""
    nodes, allocs = cluster(4000, seed=7, slots=700, zones=300)
    targets = [SpreadTarget("s%05d" % k, 1) for k in range(0, 700, 7)][:40]
    jb = job(60,
             spreads=[Spread("${node.datacenter}", 40, [SpreadTarget("dc1", 50), SpreadTarget("dc2", 30)]),
                      Spread("${meta.rack}", 30),
                      Spread("${meta.unique.slot}", 30, targets)],
             constraints=[Constraint("${meta.unique.zone}", "2", "distinct_property"),
                          Constraint("${meta.rack}", "6", "distinct_property")],
             tg_constraints=[Constraint("${node.unique.name}", "", "distinct_property")])
    re = _both(nodes, allocs, jb, synth.shuffle(len(nodes), 3))
    assert sum(1 for x in re if x.row >= 0) > 40


def test_distinct_property_with_many_values_only():
    nodes, allocs = cluster(2500, seed=9, zones=900)
    jb = job(150, constraints=[Constraint("${meta.unique.zone}", "1", "distinct_property")])
    _both(nodes, allocs, jb, synth.shuffle(len(nodes), 4))


def test_sweep_loop_with_hbm_counts():
    # a full-pass count loop over >= 8192 nodes runs as device-resident sweeps;
    # 10000 values: k_sweep_step rebuilds the table from the HBM counts
    nodes, allocs = cluster(10000, seed=11, slots=10000)
    jb = job(12, spreads=[Spread("${meta.unique.slot}", 100)])
    _both(nodes, allocs, jb, synth.shuffle(len(nodes), 5))


def test_select_protocol_with_many_values():
    from nomad_amd.stack import SelectOptions  # noqa: F401
    nodes, allocs = cluster(2000, seed=13, slots=1500)
    jb = job(30, spreads=[Spread("${meta.unique.slot}", 100)])
    perm = synth.shuffle(len(nodes), 6)
    out = []
    for cls in (OracleGenericStack, _engine):
        st = cls()
        st.SetState(nodes, allocs)
        st.SetJob(jb)
        st.SetNodes(list(perm))
        res = []
        for _ in range(30):
            r = st.Select(0)
            if r is None:
                break
            st.Commit(0, r.row)
            res.append((r.row, r.final_score, tuple(r.scores)))
        out.append(res)
    assert out[0] == out[1]


def _many_meta(nodes, keys, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    for nd in nodes:
        for k, card in keys:
            nd.meta[k] = "v%d" % int(rng.integers(0, card))
        nd.compute_class()


def test_ten_sets_against_the_oracle():
    """Five spreads and five distinct_property sets (10 > round 4's 8)."""
    nodes, allocs = cluster(3000, seed=21, slots=400)
    keys = [("p%d" % k, 3 + 2 * k) for k in range(8)]
    _many_meta(nodes, keys, 22)
    jb = job(80,
             spreads=[Spread("${meta.p0}", 30), Spread("${meta.p1}", 20, [SpreadTarget("v1", 40)]),
                      Spread("${meta.p2}", 20), Spread("${node.datacenter}", 15),
                      Spread("${meta.unique.slot}", 15)],
             constraints=[Constraint("${meta.p3}", "30", "distinct_property"),
                          Constraint("${meta.p4}", "25", "distinct_property")],
             tg_constraints=[Constraint("${meta.p5}", "20", "distinct_property"),
                             Constraint("${meta.p6}", "15", "distinct_property"),
                             Constraint("${meta.p7}", "12", "distinct_property")])
    re = _both(nodes, allocs, jb, synth.shuffle(len(nodes), 7))
    assert sum(1 for x in re if x.row >= 0) > 40


def test_sixteen_sets_and_the_limit_past_them():
    nodes, allocs = cluster(1500, seed=23)
    keys = [("q%d" % k, 4 + k) for k in range(17)]
    _many_meta(nodes, keys, 24)
    spreads = [Spread("${meta.q%d}" % k, 5 + k) for k in range(8)]
    dps = [Constraint("${meta.q%d}" % k, "40", "distinct_property") for k in range(8, 16)]
    jb = job(40, spreads=spreads, constraints=dps)
    re = _both(nodes, allocs, jb, synth.shuffle(len(nodes), 8))
    assert sum(1 for x in re if x.row >= 0) > 20
    # a 17th set is past the device tables: the engine says so
    from nomad_amd.stack import Unsupported
    jb17 = job(40, spreads=spreads, constraints=dps + [Constraint("${meta.q16}", "40", "distinct_property")])
    st = _engine()
    st.SetState(nodes, allocs)
    st.SetJob(jb17)
    st.SetNodes(list(synth.shuffle(len(nodes), 8)))
    with pytest.raises(Unsupported):
        st.Select(0)
