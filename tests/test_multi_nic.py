"""Nodes with several host network devices (multi-NIC), and allocs holding
bandwidth on a device other than their node's first.

NetworkIndex keeps bandwidth per device (AvailBandwidth / UsedBandwidth,
nomad/structs/network.go:36-43, 108-114, 196-217); AssignNetwork walks the
node's AvailNetworks in order and takes the first address whose device has
the bandwidth and whose ports are free (yieldIP, network.go:294-315,
407-482); PreemptForNetwork groups its candidates by device
(scheduler/preemption.go:270-455). The engine answers these nodes from the
host's first fit (engine.cpp build_md, TgTables::md); candidates on two
devices make the reference's answer depend on Go map order, which both sides
refuse. The reference pins one case (preemption_test.go:408,
tests/test_preemption.py); the rest is engine vs oracle on random clusters
(parity unpinned beyond the oracle's restatement).
"""
import numpy as np
import pytest

from nomad_amd import synth
from nomad_amd.stack import SelectOptions
from nomad_amd.structs import Allocation, Job, NetworkResource, SchedulerConfig, Task, TaskGroup
from oracle.oracle import OracleGenericStack, OracleSystemStack
from tests.helpers import assert_same_placements, run_place


def _engine(**kw):
    from nomad_amd.stack import GenericStack
    return GenericStack(**kw)


def nic_job(mbits, ports=(), count=1, priority=50, cpu=100, dyn=0, job_id="nic"):
    net = NetworkResource(mode="host", mbits=mbits, dynamic_ports=dyn, reserved_ports=list(ports),
                          port_labels=["p%d" % p for p in ports])
    return Job(id=job_id, priority=priority, task_groups=[TaskGroup(
        name="web", count=count, ephemeral_disk_mb=100,
        tasks=[Task(name="web", driver="exec", cpu=cpu, memory_mb=64, network=net)])])


def nic_cluster(n, seed, two_nic=0.5, absent=0.05, busy=0.0, mixed=True):
    """Nodes with eth0 and, on `two_nic` of them, eth1 (each CIDR one
    address); allocs on either device, a few on a device the node lacks;
    `busy` of the nodes hold extra low-priority allocs (eviction candidates),
    on either device (`mixed`) or on eth0 only, the others then high-priority."""
    rng = np.random.Generator(np.random.PCG64(seed))
    ids = sorted(synth.uuids(n, seed))
    nodes, allocs = [], []
    for k, nid in enumerate(ids):
        ip0 = "10.%d.%d.%d" % (k >> 16, (k >> 8) & 255, k & 255)
        ip1 = "10.%d.%d.%d" % (128 + (k >> 16), (k >> 8) & 255, k & 255)
        nd = synth.mock_node(nid)
        nd.name = "node-%05d" % k
        nd.reserved_host_ports = [9000] if rng.random() < 0.2 else []
        nets = [NetworkResource(mode="host", device="eth0", cidr=ip0 + "/32", ip=ip0,
                                mbits=int(rng.choice([600, 1000])))]
        two = rng.random() < two_nic
        if two:
            nets.append(NetworkResource(mode="host", device="eth1", cidr=ip1 + "/32", ip=ip1,
                                        mbits=int(rng.choice([400, 1000]))))
        nd.networks = nets
        nd.compute_class()
        nodes.append(nd)
        full = rng.random() < busy
        for q in range(int(rng.integers(0, 4)) + (2 if full else 0)):
            on1 = two and rng.random() < 0.5
            dev, ip = ("eth1", ip1) if on1 else ("eth0", ip0)
            if rng.random() < absent:
                dev, ip = "eth9", "172.16.0.9"
            port = int(rng.choice([8080, 443, 5000]))
            prio = int(rng.choice([20, 30, 95] if full else [50, 95]))
            if not mixed:
                prio = int(rng.choice([20, 30])) if (full and dev == "eth0") else 95
            allocs.append(Allocation(node_id=nid, job_id="svc-%d" % (k % 7 + q), task_group="web",
                                     cpu_shares=1200 if full else 200, memory_mb=128, disk_mb=50,
                                     priority=prio, net_mbits=int(rng.choice([100, 300, 600])),
                                     net_device=dev, ports=[(ip, port)] if rng.random() < 0.5 else []))
    return nodes, allocs


@pytest.mark.gpu
@pytest.mark.parametrize("mbits,ports", [(550, ()), (450, ()), (200, (8080,)), (100, (443, 5000))])
def test_multi_nic_count_loop(mbits, ports):
    """pe_place's count loop: every placement equal to the oracle's, the
    nodes' devices filling one after the other."""
    nodes, allocs = nic_cluster(1200, seed=mbits + len(ports))
    job = nic_job(mbits, ports, count=2500)
    perm = synth.shuffle(len(nodes), 4)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm)
    _, _, re = run_place(_engine, nodes, allocs, job, perm)
    assert_same_placements(re, ro)
    assert 0 < sum(1 for x in re if x.row >= 0) < 2500


@pytest.mark.gpu
@pytest.mark.parametrize("ports", [(), (8080,)])
def test_multi_nic_select_commit_metrics(ports):
    """The caller's Select / Commit loop with AllocMetric on: the maps'
    network reasons ("bandwidth exceeded", the port collision of the last
    device tried) equal the oracle's, with plan stops in between."""
    nodes, allocs = nic_cluster(300, seed=11)
    job = nic_job(350, ports, count=400)
    perm = synth.shuffle(len(nodes), 6)
    sts = []
    for cls in (OracleGenericStack, _engine):
        st = cls()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
        st.EnableMetrics(True)
        st.StopAllocs(list(range(0, len(allocs), 9)))
        sts.append(st)
    placed = 0
    for _ in range(400):
        ro, re = (st.SelectRaw(0) for st in sts)
        assert_same_placements([re], [ro])
        assert sts[1].LastMetrics() == sts[0].LastMetrics()
        if ro.row < 0:
            break
        placed += 1
        for st in sts:
            st.Commit(0, ro.row)
    assert placed > 50


def _select_or_refuse(st, opts=None):
    try:
        return st.SelectRaw(0, opts), None
    except Exception as e:   # PE_EUNSUPPORTED / oracle Unsupported
        return None, str(e)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,mixed", [(3, False), (4, False), (5, True)])
def test_multi_nic_preempt_retry(seed, mixed):
    """selectNextOption's loop (generic_sched.go:773-792) on a busy multi-NIC
    cluster: a nil Select retried with Preempt=true; the preempted sets equal
    the oracle's, and a Preempt Select whose candidates sit on two devices is
    refused on both sides (then the caller's chain would answer: the test
    stops there)."""
    nodes, allocs = nic_cluster(200, seed=seed, busy=0.8, absent=0.0, mixed=mixed)
    job = nic_job(700, (), count=150, priority=70, cpu=1500)
    cfg = SchedulerConfig(preempt_service=True)
    perm = synth.shuffle(len(nodes), 2)
    sts = []
    for cls in (OracleGenericStack, _engine):
        st = cls(config=cfg)
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
        sts.append(st)
    evicting = refused = 0
    for _ in range(150):
        ro, re = (st.SelectRaw(0) for st in sts)
        assert_same_placements([re], [ro])
        if ro.row < 0:
            (ro, eo), (re, ee) = (_select_or_refuse(st, SelectOptions(preempt=True)) for st in sts)
            assert (eo is None) == (ee is None), (eo, ee)
            if eo is not None:
                refused += 1
                break
            assert_same_placements([re], [ro])
            assert sorted(re.preempted) == sorted(ro.preempted)
            if ro.row < 0:
                break
            evicting += bool(ro.preempted)
        for st in sts:
            st.Commit(0, ro.row, ro.preempted)
    assert (refused > 0) if mixed else (evicting > 0 and refused == 0)


@pytest.mark.gpu
def test_multi_nic_system_stack():
    """SystemScheduler batch (pe_system_place) on a multi-NIC cluster."""
    from nomad_amd.stack import SystemStack
    nodes, allocs = nic_cluster(3000, seed=21)
    job = nic_job(500, (8080,), job_id="sys-nic")
    job.type = 2
    out = []
    for cls in (OracleSystemStack, SystemStack):
        st = cls()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(list(range(len(nodes))))
        out.append(st.SystemPlace(0))
    (so, to, po), (se, te, pe) = out
    assert po == pe and (to == te).all()
    m = to == 0
    assert (so[m] == se[m]).all()
    assert 0 < po < len(nodes)


def test_multi_nic_oracle_first_fit():
    """The oracle's AssignNetwork takes eth1 once eth0 is out of bandwidth,
    and the placement's bandwidth stays on eth1 for the next Select."""
    nd = synth.mock_node("n0")
    nd.networks = [NetworkResource(mode="host", device="eth0", cidr="10.0.0.1/32", mbits=1000),
                   NetworkResource(mode="host", device="eth1", cidr="10.1.0.1/32", mbits=1000)]
    nd.compute_class()
    job = nic_job(400, (), count=6)
    st, _, res = run_place(OracleGenericStack, [nd], [], job, [0], count=6)
    # 2 x 400 on eth0, 2 x 400 on eth1, then neither has 400 left
    rows = [r.row for r in res]
    assert rows[:4] == [0, 0, 0, 0] and rows[4] == -1
