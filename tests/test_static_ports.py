"""Static port asks (NetworkIndex.AssignPorts' ReservedPorts, network.go:317-363).

A task group's static port goes on the first address of its host network on
the node; it collides with the ports that address already has: the node's
own reservations for that IP (NodeNetworks address ReservedPorts), the node's
ReservedHostPorts, and the ports the proposed allocs hold on that IP
(NetworkIndex.SetNode / AddAllocs, network.go:92-193), including this plan's
earlier placements of the group. The errors are the reference's texts
("reserved port collision <label>=<port>", "no addresses available for
"<network>" network", "invalid port <n> (out of range)"). These cases restate
that code (no reference test pins a scheduler outcome of static ports:
parity unpinned beyond the restatement); engine vs oracle placement by
placement on random clusters, with plan stops, metrics and the SystemStack.
"""
import numpy as np
import pytest

from nomad_amd import synth
from nomad_amd.structs import Allocation, Job, NetworkResource, Task, TaskGroup
from oracle.oracle import OracleGenericStack, OracleSystemStack
from tests.helpers import assert_same_placements, run_place


def _engine(**kw):
    from nomad_amd.stack import GenericStack
    return GenericStack(**kw)


STACKS = [pytest.param(OracleGenericStack, id="oracle"),
          pytest.param(_engine, id="engine", marks=pytest.mark.gpu)]


def static_job(ports, labels=None, host_network="default", dyn=1, count=1, job_id="static"):
    net = NetworkResource(mode="host", dynamic_ports=dyn, reserved_ports=list(ports),
                          port_labels=list(labels or ["p%d" % p for p in ports]), host_network=host_network)
    return Job(id=job_id, task_groups=[TaskGroup(name="web", count=count, ephemeral_disk_mb=100, network=net,
                                                 tasks=[Task(name="web", driver="exec", cpu=100, memory_mb=64)])])


def _node(nid, addresses=None, reserved_host_ports=(22,)):
    n = synth.mock_node(nid)
    if addresses is not None:
        n.addresses = list(addresses)
        n.host_network_aliases = sorted({a for a, _, _ in addresses})
    n.reserved_host_ports = list(reserved_host_ports)
    n.compute_class()
    return n


@pytest.mark.parametrize("stack_cls", STACKS)
def test_static_port_reasons(stack_cls):
    nodes = [_node("n0"),
             _node("n1", [("default", "10.0.0.1", ""), ("private", "192.168.0.101", "9091-10000")]),
             _node("n2", [("default", "10.0.0.2", "")])]
    cases = [
        (static_job([22], ["ssh"]), [None, None, None], "network: reserved port collision ssh=22"),
        (static_job([8080], ["http"]), [0, 1, 2], None),
        # nodes without the host network are filtered by the NetworkChecker first
        (static_job([9500], ["admin"], host_network="private"), [None, None, None], None),
        (static_job([10001], ["admin"], host_network="private"), [None, 1, None], None),
        (static_job([70000], ["big"]), [None, None, None], "network: invalid port 70000 (out of range)"),
    ]
    for job, want, reason in cases:
        for row, w in enumerate(want):
            # a fresh stack per node: the FeasibilityWrapper memoises the network
            # checker per ComputedClass, which these nodes share
            st = stack_cls()
            st.SetState(nodes, [])
            st.SetJob(job)
            st.EnableMetrics(True)
            st.SetNodes([row])
            r = st.SelectRaw(0)
            assert (r.row if r.row >= 0 else None) == w, (job.task_groups[0].network.reserved_ports, row)
            if w is None and reason and row == 0:
                assert st.LastMetrics()["DimensionExhausted"] == {reason: 1}
    # the private address reserves 9091-10000
    st = stack_cls()
    st.SetState(nodes, [])
    st.SetJob(static_job([9500], ["admin"], host_network="private"))
    st.EnableMetrics(True)
    st.SetNodes([1])
    assert st.SelectRaw(0).row == -1
    assert st.LastMetrics()["DimensionExhausted"] == {"network: reserved port collision admin=9500": 1}


@pytest.mark.parametrize("stack_cls", STACKS)
def test_static_port_held_by_allocs_and_own_placements(stack_cls):
    nodes = [_node("n0"), _node("n1")]
    allocs = [Allocation(node_id="n0", job_id="other", task_group="web", cpu_shares=100, memory_mb=64,
                         ports=[("192.168.0.100", 8080)])]
    st = stack_cls()
    st.SetState(nodes, allocs)
    st.SetJob(static_job([8080], ["http"], count=3))
    st.SetNodes([0, 1])
    r = st.SelectRaw(0)
    assert r.row == 1                      # n0's address already holds 8080
    st.Commit(0, r.row)
    assert st.SelectRaw(0).row == -1       # the placement on n1 holds it now
    st.StopAllocs([0])                     # the other job's alloc leaves n0 in this plan
    st.SetNodes([0, 1])
    assert st.SelectRaw(0).row == 0


def port_cluster(n, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    ids = sorted(synth.uuids(n, seed))
    nodes, allocs = [], []
    for k, nid in enumerate(ids):
        ip = "10.%d.%d.%d" % (k >> 16, (k >> 8) & 255, k & 255)
        addrs = [("default", ip, "22,9000-9010" if rng.random() < 0.1 else "")]
        if rng.random() < 0.5:
            addrs.append(("private", "172.16.%d.%d" % ((k >> 8) & 255, k & 255), ""))
        nd = _node(nid, addrs, reserved_host_ports=(22,) if rng.random() < 0.5 else ())
        nd.name = "node-%05d" % k
        nd.compute_class()
        nodes.append(nd)
        for _ in range(int(rng.integers(0, 3))):
            port = int(rng.choice([8080, 25000, 443, 5000]))
            allocs.append(Allocation(node_id=nid, job_id="svc-%d" % (k % 7), task_group="web", cpu_shares=200,
                                     memory_mb=128, disk_mb=50, dyn_ports=int(20000 <= port <= 32000),
                                     ports=[(ip, port)]))
    return nodes, allocs


@pytest.mark.gpu
@pytest.mark.parametrize("n,count,ports", [(800, 300, [8080]), (3000, 500, [8080, 25000]), (12000, 400, [443])])
def test_static_ports_count_loop(n, count, ports):
    nodes, allocs = port_cluster(n, seed=n)
    job = static_job(ports, count=count)
    perm = synth.shuffle(len(nodes), 5)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm)
    _, _, re = run_place(_engine, nodes, allocs, job, perm)
    assert_same_placements(re, ro)
    assert sum(1 for x in re if x.row >= 0) > 0


@pytest.mark.gpu
def test_static_ports_select_commit_stops_and_metrics():
    nodes, allocs = port_cluster(600, seed=31)
    job = static_job([8080], count=100)
    perm = synth.shuffle(len(nodes), 6)
    sts = []
    for cls in (OracleGenericStack, _engine):
        st = cls()
        st.SetState(nodes, allocs)
        st.SetJob(job)
        st.SetNodes(perm)
        st.EnableMetrics(True)
        st.StopAllocs([i for i, a in enumerate(allocs) if a.ports and a.ports[0][1] == 8080][:40])
        sts.append(st)
    for _ in range(100):
        ro, re = (st.SelectRaw(0) for st in sts)
        assert_same_placements([re], [ro])
        assert sts[1].LastMetrics() == sts[0].LastMetrics()
        if ro.row < 0:
            break
        for st in sts:
            st.Commit(0, ro.row)


@pytest.mark.gpu
def test_static_ports_system_stack():
    from nomad_amd.stack import SystemStack
    nodes, allocs = port_cluster(2000, seed=8)
    job = static_job([8080], job_id="sys-static")
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


# ---- task network static ports (AssignNetwork, network.go:407-442) and
# PreemptForNetwork's reserved-port step (preemption.go:302-342) ------------

def task_static_job(ports, mbits=10, dyn=0, count=1, job_id="tstatic", priority=50, cpu=100):
    net = NetworkResource(mode="host", mbits=mbits, dynamic_ports=dyn, reserved_ports=list(ports),
                          port_labels=["p%d" % p for p in ports])
    return Job(id=job_id, priority=priority, task_groups=[TaskGroup(
        name="web", count=count, ephemeral_disk_mb=100,
        tasks=[Task(name="web", driver="exec", cpu=cpu, memory_mb=64, network=net)])])


def task_port_cluster(n, seed, busy=0.0):
    """Nodes whose eth0 CIDR is the node's one address (yieldIP), allocs holding
    static ports and bandwidth on it; `busy` of the nodes nearly full of
    low-priority work (preemption candidates)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    ids = sorted(synth.uuids(n, seed))
    nodes, allocs = [], []
    for k, nid in enumerate(ids):
        ip = "10.%d.%d.%d" % (k >> 16, (k >> 8) & 255, k & 255)
        nd = _node(nid, [("default", ip, "22" if rng.random() < 0.2 else "")],
                   reserved_host_ports=(9000,) if rng.random() < 0.3 else ())
        nd.networks = [NetworkResource(mode="host", device="eth0", cidr=ip + "/32", mbits=1000)]
        nd.name = "node-%05d" % k
        nd.compute_class()
        nodes.append(nd)
        full = rng.random() < busy
        for q in range(int(rng.integers(0, 3)) + (2 if full else 0)):
            port = int(rng.choice([8080, 443, 5000, 9000]))
            prio = int(rng.choice([20, 30, 95] if full else [50, 95]))
            allocs.append(Allocation(node_id=nid, job_id="svc-%d" % (k % 7 + q), task_group="web",
                                     cpu_shares=1600 if full else 200, memory_mb=128, disk_mb=50,
                                     priority=prio, net_mbits=int(rng.choice([50, 300, 600])),
                                     ports=[(ip if rng.random() < 0.8 else "172.16.0.1", port)]))
    return nodes, allocs


@pytest.mark.parametrize("stack_cls", STACKS)
def test_task_static_port_reasons(stack_cls):
    """mock.Node(): the address 192.168.0.100 is the CIDR's one address, so
    ReservedHostPorts 22 collides on it; a port held by an alloc on that IP
    collides, one held on another IP does not; invalid ports fail; bandwidth
    is checked before the ports."""
    nodes = [_node("n0"), _node("n1"), _node("n2")]
    allocs = [Allocation(node_id="n1", job_id="other", task_group="web", cpu_shares=100, memory_mb=64,
                         ports=[("192.168.0.100", 8080)], net_mbits=10),
              Allocation(node_id="n2", job_id="other", task_group="web", cpu_shares=100, memory_mb=64,
                         ports=[("10.9.9.9", 8080)], net_mbits=10)]
    cases = [
        (task_static_job([22]), [None, None, None], "network: reserved port collision p22=22"),
        (task_static_job([8080]), [0, None, 2], "network: reserved port collision p8080=8080"),
        (task_static_job([70000]), [None, None, None], "network: invalid port 70000 (out of range)"),
        (task_static_job([8080], mbits=2000), [None, None, None], "network: bandwidth exceeded"),
    ]
    for job, want, reason in cases:
        for row, w in enumerate(want):
            st = stack_cls()
            st.SetState(nodes, allocs)
            st.SetJob(job)
            st.EnableMetrics(True)
            st.SetNodes([row])
            r = st.SelectRaw(0)
            assert (r.row if r.row >= 0 else None) == w, (job.task_groups[0].tasks[0].network.reserved_ports, row)
            if w is None and reason and row in (0, 1) and "p8080" not in reason:
                assert st.LastMetrics()["DimensionExhausted"] == {reason: 1}
            if w is None and "p8080" in reason:
                assert st.LastMetrics()["DimensionExhausted"] == {reason: 1}


@pytest.mark.gpu
@pytest.mark.parametrize("n,count,ports", [(900, 900, [8080]), (4000, 3000, [443, 5000])])
def test_task_static_ports_count_loop(n, count, ports):
    nodes, allocs = task_port_cluster(n, seed=n)
    job = task_static_job(ports, count=count)
    perm = synth.shuffle(len(nodes), 3)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm)
    _, _, re = run_place(_engine, nodes, allocs, job, perm)
    assert_same_placements(re, ro)
    assert 0 < sum(1 for x in re if x.row >= 0) < count


@pytest.mark.gpu
@pytest.mark.parametrize("task", [True, False])
def test_static_port_preemption_count_loop(task):
    """Saturated cluster, preemption on: nil Selects retried with Preempt=true
    evict the static port's holders (and bandwidth for task networks),
    placement by placement equal to the oracle, with the preempted sets."""
    from nomad_amd.structs import SchedulerConfig
    nodes, allocs = task_port_cluster(1500, seed=77, busy=0.9)
    if task:
        job = task_static_job([8080], mbits=500, count=400, priority=70, cpu=1500)
    else:
        job = static_job([8080], dyn=0, count=400)
        job.priority = 70
        job.task_groups[0].tasks[0].cpu = 1500
    cfg = SchedulerConfig(preempt_service=True)
    perm = synth.shuffle(len(nodes), 9)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm, config=cfg)
    _, _, re = run_place(_engine, nodes, allocs, job, perm, config=cfg)
    assert_same_placements(re, ro)
    assert [sorted(x.preempted) for x in re] == [sorted(x.preempted) for x in ro]
    assert sum(1 for x in re if x.preempted) > 5


def wide_port_cluster(n, seed):
    """task_port_cluster's nodes with 36-70 small allocs each on the busy ones,
    the static port's holder anywhere in the node's list (often past slot 32)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    ids = sorted(synth.uuids(n, seed))
    nodes, allocs = [], []
    for k, nid in enumerate(ids):
        ip = "10.%d.%d.%d" % (k >> 16, (k >> 8) & 255, k & 255)
        nd = _node(nid, [("default", ip, "")], reserved_host_ports=())
        nd.networks = [NetworkResource(mode="host", device="eth0", cidr=ip + "/32", mbits=1000)]
        nd.name = "node-%05d" % k
        nd.compute_class()
        nodes.append(nd)
        m = int(rng.integers(36, 71)) if rng.random() < 0.85 else int(rng.integers(0, 4))
        holder = int(rng.integers(0, m)) if m else -1
        for q in range(m):
            ports = []
            if q == holder or rng.random() < 0.05:
                ports = [(ip, int(rng.choice([8080, 8080, 443])))]
            allocs.append(Allocation(node_id=nid, job_id="svc-%d" % (q % 9), task_group="web",
                                     cpu_shares=3700 // max(m, 1), memory_mb=64, disk_mb=20,
                                     priority=int(rng.choice([20, 30, 95], p=[0.45, 0.45, 0.1])),
                                     net_mbits=int(rng.choice([5, 10, 20])), ports=ports))
    return nodes, allocs


@pytest.mark.gpu
@pytest.mark.parametrize("task", [True, False])
def test_static_port_preemption_on_wide_nodes(task):
    """Static-port preemption on nodes of 36-70 allocs (the holder past slot 32
    on most): the blocker list is indices, not the first 32 slots' bits.
    Engine vs oracle, preempted sets included."""
    from nomad_amd.structs import SchedulerConfig
    nodes, allocs = wide_port_cluster(400, seed=91)
    if task:
        job = task_static_job([8080], mbits=30, count=150, priority=70, cpu=1500)
    else:
        job = static_job([8080], dyn=0, count=150)
        job.priority = 70
        job.task_groups[0].tasks[0].cpu = 1500
    cfg = SchedulerConfig(preempt_service=True)
    perm = synth.shuffle(len(nodes), 10)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm, config=cfg)
    _, _, re = run_place(_engine, nodes, allocs, job, perm, config=cfg)
    assert_same_placements(re, ro)
    assert [sorted(x.preempted) for x in re] == [sorted(x.preempted) for x in ro]
    assert sum(1 for x in re if x.preempted and any(p >= 0 for p in x.preempted)) > 5
