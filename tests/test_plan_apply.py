"""Plan applier fit check: evaluatePlanPlacements /
evaluateNodePlan → AllocsFit(checkDevices=true).

CPU tests pin the oracle (oracle/plan_apply.py) against the reference's own
tests, nomad/plan_apply_test.go:392-987 (TestPlanApply_EvalPlan_* and
TestPlanApply_EvalNodePlan_*), plus ParsePortRanges and SetNode corner cases.
GPU tests run the HIP planner (pe_planner_*) on the same cases and on seeded
random snapshots, bit-exact per node against the oracle, including
commit chains (a plan applied, the next evaluated against the result).
"""
import copy
import random

import numpy as np
import pytest

from nomad_amd import abi
from nomad_amd.plan import (AllocDevice, AllocNetwork, NodeNetworkAddress, Plan, PlanAlloc, PlanNode, Port,
                            assemble_result)
from nomad_amd.synth_plan import full_node_alloc, mock_alloc, mock_node, nvidia_node, random_case, system_plan
from oracle import plan_apply as O

NODE1 = "9e1d3f0c-1111-4f1b-9d7e-000000000001"
NODE2 = "9e1d3f0c-2222-4f1b-9d7e-000000000002"


def _rng_id(i):
    return "a1a1a1a1-0000-4000-8000-%012d" % i


# ---- reference KATs (plan_apply_test.go) -------------------------------------
# Each returns (nodes, snapshot allocs, plan, expected {node_id: (fit, reason or None=any non-empty)}).


def kat_eval_plan_simple():                      # :392-434
    node = mock_node(NODE1)
    return [node], [], Plan(node_allocation={NODE1: [mock_alloc(_rng_id(1))]}), {NODE1: (True, "")}


def kat_eval_plan_preemption():                  # :436-548
    node = mock_node(NODE1)
    node.cpu_shares, node.memory_mb, node.disk_mb = 2000, 4192, 30 * 1024
    node.networks = [("eth0", "")]
    node.addresses = []
    pre = mock_alloc(_rng_id(1), NODE1)
    pre.cpu_shares, pre.memory_mb, pre.disk_mb = 1500, 4000, 25 * 1024
    new = mock_alloc(_rng_id(2), NODE1)
    new.cpu_shares, new.memory_mb, new.disk_mb = 1500, 3200, 24 * 1024
    plan = Plan(node_allocation={NODE1: [new]}, node_preemptions={NODE1: [pre]})
    return [node], [pre], plan, {NODE1: (True, "")}


def kat_eval_plan_partial(all_at_once=False):    # :550-657
    n1, n2 = mock_node(NODE1), mock_node(NODE2)
    a1 = mock_alloc(_rng_id(1))
    a2 = full_node_alloc(_rng_id(2), n2)          # does not fit: 4000 > 4000 - 100
    plan = Plan(node_allocation={NODE1: [a1], NODE2: [a2]}, all_at_once=all_at_once)
    return [n1, n2], [], plan, {NODE1: (True, ""), NODE2: (False, "cpu")}


def kat_node_simple():                           # :659-684
    return [mock_node(NODE1)], [], Plan(node_allocation={NODE1: [mock_alloc(_rng_id(1))]}), {NODE1: (True, "")}


def kat_node_not_ready():                        # :686-712
    n = mock_node(NODE1)
    n.status = "initializing"
    return [n], [], Plan(node_allocation={NODE1: [mock_alloc(_rng_id(1))]}), \
        {NODE1: (False, "node is not ready for placements")}


def kat_node_drain():                            # :714-739 (mock.DrainNode ⇒ ineligible)
    n = mock_node(NODE1)
    n.scheduling_eligibility = "ineligible"
    return [n], [], Plan(node_allocation={NODE1: [mock_alloc(_rng_id(1))]}), {NODE1: (False, "node is not eligible")}


def kat_node_not_exist():                        # :741-765
    ghost = "12345678-abcd-efab-cdef-123456789abc"
    return [], [], Plan(node_allocation={ghost: [mock_alloc(_rng_id(1))]}), {ghost: (False, "node does not exist")}


def _reserved_nil(n):
    n.reserved_cpu = n.reserved_memory_mb = n.reserved_disk_mb = 0
    n.reserved_host_ports = ""
    return n


def kat_node_full():                             # :767-802
    n = _reserved_nil(mock_node(NODE1))
    a = full_node_alloc(_rng_id(1), n)
    return [n], [a], Plan(node_allocation={NODE1: [mock_alloc(_rng_id(2), NODE1)]}), {NODE1: (False, "cpu")}


def kat_node_full_device():                      # :804-855
    inst = ["6e3c1c3c-0000-4000-8000-00000000000%d" % k for k in range(2)]
    n = _reserved_nil(nvidia_node(NODE1, inst))
    a = mock_alloc(_rng_id(1), NODE1)
    a.devices = [AllocDevice("nvidia", "gpu", "1080ti", [inst[0]])]
    a2 = mock_alloc(_rng_id(2), NODE1)
    a2.task_networks = {"web": []}
    a2.devices = [AllocDevice("nvidia", "gpu", "1080ti", [inst[0]])]
    return [n], [a], Plan(node_allocation={NODE1: [a2]}), {NODE1: (False, "device oversubscribed")}


def kat_node_update_existing():                  # :857-887
    n = _reserved_nil(mock_node(NODE1))
    a = full_node_alloc(_rng_id(1), n)
    return [n], [a], Plan(node_allocation={NODE1: [copy.deepcopy(a)]}), {NODE1: (True, "")}


def kat_node_full_evict():                       # :889-925
    n = _reserved_nil(mock_node(NODE1))
    a = full_node_alloc(_rng_id(1), n)
    ev = copy.deepcopy(a)
    ev.desired_status = "evict"
    plan = Plan(node_update={NODE1: [ev]}, node_allocation={NODE1: [mock_alloc(_rng_id(2), NODE1)]})
    return [n], [a], plan, {NODE1: (True, "")}


def kat_node_full_alloc_evict():                 # :927-958
    n = _reserved_nil(mock_node(NODE1))
    a = full_node_alloc(_rng_id(1), n)
    a.desired_status = "evict"
    return [n], [a], Plan(node_allocation={NODE1: [mock_alloc(_rng_id(2), NODE1)]}), {NODE1: (True, "")}


def kat_node_down_evict_only():                  # :960-987
    n = _reserved_nil(mock_node(NODE1))
    n.status = "down"
    a = full_node_alloc(_rng_id(1), n)
    ev = copy.deepcopy(a)
    ev.desired_status = "evict"
    return [n], [a], Plan(node_update={NODE1: [ev]}), {NODE1: (True, "")}


# nomad/structs/funcs_test.go AllocsFit cases, as a snapshot alloc plus a
# plan placing a copy (proposed = [a, a'], which is what AllocsFit receives).

def _allocsfit_node(cores=True):
    n = PlanNode(id=NODE1, cpu_shares=2000, memory_mb=2048, disk_mb=10000, reserved_cpu=1000,
                 reserved_memory_mb=1024, reserved_disk_mb=5000, networks=[("eth0", "")],
                 addresses=[NodeNetworkAddress("10.0.0.1")], reserved_host_ports="80")
    if cores:
        n.reservable_cores = [0, 1]
    return n


def kat_allocsfit_twice():                       # TestAllocsFit :266-356 (a1, a1 ⇒ no fit)
    a = PlanAlloc(id=_rng_id(1), node_id=NODE1, cpu_shares=1000, memory_mb=1024, disk_mb=5000,
                  shared_ports=[Port(8000, "10.0.0.1")])
    b = copy.deepcopy(a)
    b.id = _rng_id(2)
    return [_allocsfit_node()], [a], Plan(node_allocation={NODE1: [b]}), {NODE1: (False, "cpu")}


def kat_allocsfit_once():                        # TestAllocsFit :348-353 (a1 alone fits)
    a = PlanAlloc(id=_rng_id(1), node_id=NODE1, cpu_shares=1000, memory_mb=1024, disk_mb=5000,
                  shared_ports=[Port(8000, "10.0.0.1")])
    return [_allocsfit_node()], [], Plan(node_allocation={NODE1: [a]}), {NODE1: (True, "")}


def kat_allocsfit_cores():                       # TestAllocsFit :358-405 (a2, a2 ⇒ "cores")
    a = PlanAlloc(id=_rng_id(1), node_id=NODE1, cpu_shares=500, memory_mb=512, disk_mb=1000, reserved_cores=[0])
    b = copy.deepcopy(a)
    b.id = _rng_id(2)
    return [_allocsfit_node()], [a], Plan(node_allocation={NODE1: [b]}), {NODE1: (False, "cores")}


def kat_allocsfit_terminal():                    # TestAllocsFit_TerminalAlloc :407-488
    n = _allocsfit_node(cores=False)
    n.networks = [("eth0", "10.0.0.1")]
    n.addresses = []
    a = PlanAlloc(id=_rng_id(1), node_id=NODE1, cpu_shares=1000, memory_mb=1024, disk_mb=5000,
                  task_networks={"web": [AllocNetwork(ip="10.0.0.1", device="eth0", mbits=50,
                                                      reserved_ports=[8000])]})
    b = copy.deepcopy(a)
    b.id = _rng_id(2)
    b.desired_status = "stop"
    return [n], [a], Plan(node_allocation={NODE1: [b]}), {NODE1: (True, "")}


def kat_allocsfit_devices():                     # TestAllocsFit_Devices :490-555 (checkDevices=true)
    inst = ["6e3c1c3c-0000-4000-8000-00000000000%d" % k for k in range(2)]
    n = nvidia_node(NODE1, inst)
    a = PlanAlloc(id=_rng_id(1), node_id=NODE1, cpu_shares=1000, memory_mb=1024, disk_mb=5000,
                  devices=[AllocDevice("nvidia", "gpu", "1080ti", [inst[0]])])
    b = copy.deepcopy(a)
    b.id = _rng_id(2)
    return [n], [a], Plan(node_allocation={NODE1: [b]}), {NODE1: (False, "device oversubscribed")}


KATS = [kat_allocsfit_twice, kat_allocsfit_once, kat_allocsfit_cores, kat_allocsfit_terminal, kat_allocsfit_devices,
        kat_eval_plan_simple, kat_eval_plan_preemption, kat_eval_plan_partial, kat_node_simple, kat_node_not_ready,
        kat_node_drain, kat_node_not_exist, kat_node_full, kat_node_full_device, kat_node_update_existing,
        kat_node_full_evict, kat_node_full_alloc_evict, kat_node_down_evict_only]


@pytest.mark.parametrize("kat", KATS, ids=lambda f: f.__name__)
def test_oracle_reference_kats(kat):
    nodes, allocs, plan, expect = kat()
    snap = O.Snapshot(nodes, allocs)
    for nid, (fit, why) in expect.items():
        assert O.evaluate_node_plan(snap, plan, nid) == (fit, why), nid


def test_oracle_eval_plan_results():
    # TestPlanApply_EvalPlan_Simple / _Preemption: result maps equal the plan's
    for kat in (kat_eval_plan_simple, kat_eval_plan_preemption):
        nodes, allocs, plan, _ = kat()
        snap = O.Snapshot(nodes, allocs)
        ids, fits, why = O.evaluate_plan_placements(snap, plan)
        res = assemble_result(plan, ids, fits, why, snap.alloc_by_id)
        assert res.node_allocation == plan.node_allocation
        assert res.node_preemptions == plan.node_preemptions
        assert not res.partial_commit
    # _Partial: node1 kept, node2 dropped, partial commit
    nodes, allocs, plan, _ = kat_eval_plan_partial()
    snap = O.Snapshot(nodes, allocs)
    res = assemble_result(plan, *O.evaluate_plan_placements(snap, plan), snap.alloc_by_id)
    assert NODE1 in res.node_allocation and NODE2 not in res.node_allocation and res.partial_commit
    # _Partial_AllAtOnce: nothing applied
    nodes, allocs, plan, _ = kat_eval_plan_partial(all_at_once=True)
    snap = O.Snapshot(nodes, allocs)
    res = assemble_result(plan, *O.evaluate_plan_placements(snap, plan), snap.alloc_by_id)
    assert res.node_allocation is None and res.node_update is None and res.partial_commit


def test_parse_port_ranges():
    # funcs.go:495-548 restated (no reference test pins ParsePortRanges directly)
    assert O.parse_port_ranges("") == []
    assert O.parse_port_ranges("80") == [80]
    assert O.parse_port_ranges("80,100-102, 22") == [22, 80, 100, 101, 102]
    assert O.parse_port_ranges("80,80") == [80]
    for bad in ("80,", "1-2-3", "5-3", "abc", "-1", "+5", ","):
        with pytest.raises(ValueError):
            O.parse_port_ranges(bad)


def test_setnode_collide_is_assigned_not_ored():
    # network.go:121-133: an address collision is forgotten when the
    # ReservedHostPorts step runs and finds none.
    n = mock_node(NODE1)
    n.addresses = [NodeNetworkAddress("10.0.0.1", reserved_ports="80"),
                   NodeNetworkAddress("10.0.0.1", reserved_ports="80-81")]
    n.reserved_host_ports = ""
    assert O.NetworkIndex().set_node(n) is True     # 80 twice on one IP
    n.reserved_host_ports = "22"
    assert O.NetworkIndex().set_node(n) is False    # range "22" collides nowhere: collide reassigned
    n.reserved_host_ports = "81"
    assert O.NetworkIndex().set_node(n) is True     # 81 already held by the address
    n.reserved_host_ports = "bad"
    assert O.NetworkIndex().set_node(n) is False    # parse error ⇒ collide = false
    n.reserved_host_ports = "70000"
    assert O.NetworkIndex().set_node(n) is True     # port >= maxValidPort


# ---- GPU: the HIP planner -----------------------------------------------------

def _planner():
    from nomad_amd.plan import Planner
    return Planner()


def _codes_to_pairs(codes):
    return [(int(c) == abi.PE_PLAN_FIT, abi.PLAN_REASONS[int(c)]) for c in codes]


@pytest.mark.gpu
@pytest.mark.parametrize("kat", KATS, ids=lambda f: f.__name__)
def test_planner_reference_kats(kat):
    nodes, allocs, plan, expect = kat()
    pl = _planner()
    pl.set_state(nodes, allocs)
    for nid, (fit, why) in expect.items():
        assert pl.evaluate_node_plan(plan, nid) == (fit, why), nid
    res = pl.evaluate_plan_placements(plan)
    snap = O.Snapshot(nodes, allocs)
    ref = assemble_result(plan, *O.evaluate_plan_placements(snap, plan), snap.alloc_by_id)
    assert res == ref


def _check_random(seed, **kw):
    nodes, allocs, plan = random_case(seed, **kw)
    pl = _planner()
    pl.set_state(nodes, allocs)
    ep = pl.encode(plan)
    got = _codes_to_pairs(pl.evaluate(ep))
    snap = O.Snapshot(nodes, allocs)
    ids, fits, why = O.evaluate_plan_placements(snap, plan)
    assert ids == ep.node_ids
    assert got == list(zip(fits, why)), seed
    return got


@pytest.mark.gpu
def test_planner_random_parity():
    seen = set()
    for seed in range(120):
        for fit, why in _check_random(seed):
            seen.add(why)
    # the generator reaches every reason the reference can produce
    assert {"", "node does not exist", "node is not ready for placements", "node is not eligible", "cores", "cpu",
            "memory", "disk", "reserved port collision", "device oversubscribed"} <= seen, seen


@pytest.mark.gpu
def test_planner_scratch_path_parity():
    # nodes with 600 reservable cores exceed the wave's 512-key LDS buffer
    for seed in range(200, 220):
        _check_random(seed, n_nodes=16, max_allocs=6, big_keys=True)


@pytest.mark.gpu
def test_planner_commit_chain():
    # planApply: each plan is evaluated against the snapshot with the previous
    # plan results applied (plan_apply.go:207, UpsertPlanResults).
    rng = random.Random(7)
    nodes, allocs, plan = random_case(1000, n_nodes=32)
    pl = _planner()
    pl.set_state(nodes, allocs)
    snap = O.Snapshot(nodes, allocs)
    for step in range(6):
        res = pl.evaluate_plan_placements(plan)
        ref = assemble_result(plan, *O.evaluate_plan_placements(snap, plan), snap.alloc_by_id)
        assert res == ref, step
        pl.apply(plan, res)
        snap.apply(plan, ref)
        # next plan: fresh placements on the same cluster, updates of live allocs
        _, _, plan = random_case(2000 + step, n_nodes=32)
        live = list(snap.by_id.values())
        plan = Plan()
        for n in rng.sample(nodes, 20):
            mine = [a for a in live if a.node_id == n.id]
            placed = [PlanAlloc(id="s%d-%s" % (step, n.id), node_id=n.id, cpu_shares=rng.choice([500, 1500]),
                                memory_mb=256, disk_mb=150)]
            if mine and rng.random() < 0.4:
                plan.node_update[n.id] = [rng.choice(mine)]
            plan.node_allocation[n.id] = placed
    assert pl.lib.pe_planner_snapshot_allocs(pl.h) == len(pl.allocs)


@pytest.mark.gpu
def test_planner_system_plan_properties():
    # full-size bench workload shape at 20k nodes: every fit decision matches
    # the oracle on a 2k-node prefix; the whole plan's fit count is stable
    # under re-evaluation (idempotent, no state change without commit).
    nodes, allocs, plan = system_plan(20000, seed=3)
    pl = _planner()
    pl.set_state(nodes, allocs)
    ep = pl.encode(plan)
    a = pl.evaluate(ep).copy()
    b = pl.evaluate(ep)
    assert np.array_equal(a, b)
    snap = O.Snapshot(nodes, allocs)
    for i, nid in enumerate(ep.node_ids[:2000]):
        assert _codes_to_pairs([a[i]])[0] == O.evaluate_node_plan(snap, plan, nid), nid
    assert (a == abi.PE_PLAN_FIT).mean() > 0.8


# ---- committed golden vectors (tools/make_plan_golden.py) ----------------------

def _golden():
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "plan_apply.json")
    return json.load(open(path))


def test_oracle_matches_golden():
    g = _golden()
    for seed, want in g["random_case"].items():
        nodes, allocs, plan = random_case(int(seed))
        ids, fits, why = O.evaluate_plan_placements(O.Snapshot(nodes, allocs), plan)
        assert [list(x) for x in zip(ids, fits, why)] == want, seed
    sp = g["system_plan"]
    nodes, allocs, plan = system_plan(sp["n"], sp["seed"])
    ids, fits, why = O.evaluate_plan_placements(O.Snapshot(nodes, allocs), plan)
    assert [list(x) for x in zip(ids, fits, why)] == sp["outcomes"]


@pytest.mark.gpu
def test_planner_matches_golden():
    g = _golden()
    pl = _planner()
    for seed, want in g["random_case"].items():
        nodes, allocs, plan = random_case(int(seed))
        pl.set_state(nodes, allocs)
        ep = pl.encode(plan)
        got = [[nid, f, w] for nid, (f, w) in zip(ep.node_ids, _codes_to_pairs(pl.evaluate(ep)))]
        assert got == want, seed
    sp = g["system_plan"]
    nodes, allocs, plan = system_plan(sp["n"], sp["seed"])
    pl.set_state(nodes, allocs)
    ep = pl.encode(plan)
    got = [[nid, f, w] for nid, (f, w) in zip(ep.node_ids, _codes_to_pairs(pl.evaluate(ep)))]
    assert got == sp["outcomes"]


@pytest.mark.gpu
def test_planner_incremental_commit_and_compaction():
    # commits append chunks per node; once the append room is used up the pool
    # is compacted. Every evaluation in between equals the oracle.
    nodes, allocs, plan = system_plan(3000, seed=21)
    pl = _planner()
    pl.set_state(nodes, allocs)
    snap = O.Snapshot(nodes, allocs)
    for step in range(4):
        res = pl.evaluate_plan_placements(plan)
        ref = assemble_result(plan, *O.evaluate_plan_placements(snap, plan), snap.alloc_by_id)
        assert res == ref, step
        pl.apply(plan, res)
        snap.apply(plan, ref)
        # next plan: another system alloc per node (ports move on), and every
        # third node stops one of its allocs
        nxt = Plan()
        for i, nd in enumerate(nodes):
            mine = snap.by_node.get(nd.id, [])
            a = PlanAlloc(id="%s-s%d" % (nd.id, step), node_id=nd.id, cpu_shares=250, memory_mb=128, disk_mb=150,
                          shared_ports=[Port(21000 + 7 * step + i % 5, nd.addresses[0].address)])
            nxt.node_allocation[nd.id] = [a]
            if mine and i % 3 == 0:
                nxt.node_update[nd.id] = [mine[0]]
        plan = nxt
    assert pl.lib.pe_planner_snapshot_allocs(pl.h) == len(pl.allocs)


@pytest.mark.gpu
def test_planner_threaded_flatten_matches_serial(monkeypatch):
    """The plan's flattening runs in per-worker parts (contiguous plan node
    ranges, offsets made global afterwards); with one worker it is the serial
    loop. Same codes and the same algorithmic bytes either way, with removals
    (node_update of live allocs) spread over every part, and against the
    oracle on nodes taken from every part."""
    nodes, allocs, plan = system_plan(12000, seed=17)
    snap = O.Snapshot(nodes, allocs)
    rng = random.Random(5)
    for nd in rng.sample(nodes, 3000):
        mine = snap.by_node.get(nd.id, [])
        if mine:
            plan.node_update[nd.id] = [mine[0]]
    got = []
    for threads in ("1", "5", "16"):
        monkeypatch.setenv("PE_PLAN_THREADS", threads)
        pl = _planner()
        pl.set_state(nodes, allocs)
        ep = pl.encode(plan)
        got.append((pl.evaluate(ep).copy(), pl.last_bytes()))
        pl.close()
    for codes, nbytes in got[1:]:
        assert np.array_equal(codes, got[0][0])
        assert nbytes == got[0][1]
    for i in range(0, len(ep.node_ids), 97):
        nid = ep.node_ids[i]
        assert _codes_to_pairs([got[2][0][i]])[0] == O.evaluate_node_plan(snap, plan, nid), nid
