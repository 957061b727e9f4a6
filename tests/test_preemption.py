"""Preemption: BinPack with eviction (Preemptor.PreemptForTaskGroup /
PreemptForDevice, scheduler/preemption.go:194-601) and the
PreemptionScoringIterator score (rank.go:773-844).

Known-answer tests are the reference's TestPreemption cases
(scheduler/preemption_test.go:286-1324), rebuilt at the Stack boundary: one
node, Select with Preempt=true, the set of preempted allocs. createAlloc gives
allocs cpu / memory (and task networks) but no shared disk, and the ask has an
empty EphemeralDisk, so disk is 0 on both sides. The cases whose ask holds a
static port ("No preemption because existing allocs are not low priority",
"Preempting low priority allocs not enough ...", "preemption impossible -
static port ...", "one alloc meets static port need ...", "alloc that meets
static port need ...") ask static ports in a task network (AssignNetwork's
ReservedPorts and PreemptForNetwork's reserved-port step); "preempt only from
device that has allocation with unused reserved port" runs on a node with two
network devices (test_preempt_only_from_device_with_unused_reserved_port).
"""
import math

import pytest

from nomad_amd import synth
from nomad_amd.stack import SelectOptions
from nomad_amd.structs import (Allocation, DeviceGroup, Job, NetworkResource, RequestedDevice,
                               SchedulerConfig, Task, TaskGroup)
from oracle.oracle import OracleGenericStack
from tests.helpers import assert_same_placements, run_place


def _engine(**kw):
    from nomad_amd.stack import GenericStack
    return GenericStack(**kw)


STACKS = [pytest.param(OracleGenericStack, id="oracle"),
          pytest.param(_engine, id="engine", marks=pytest.mark.gpu)]

LOW, LOW2, HIGH = 30, 40, 100


def preemption_node():
    """preemption_test.go:174-284: 4000 cpu / 8192 MB, reserved 100 / 256, eth0
    1000 MBits, 1080ti x4, 2080ti x5, F100 fpga (1 of 2 healthy)."""
    nd = synth.mock_node("node-0")
    nd.cpu_shares, nd.memory_mb, nd.disk_mb = 4000, 8192, 100 * 1024
    nd.reserved_cpu, nd.reserved_memory_mb, nd.reserved_disk_mb = 100, 256, 4 * 1024
    nd.reserved_host_ports = []
    attrs = {"memory": (11, "GiB"), "cuda_cores": 3584, "graphics_clock": (1480, "MHz"),
             "memory_bandwidth": (11, "GB/s")}
    nd.devices = [DeviceGroup("nvidia", "gpu", "1080ti", 4, dict(attrs)),
                  DeviceGroup("nvidia", "gpu", "2080ti", 5, dict(attrs)),
                  DeviceGroup("intel", "fpga", "F100", 1, {"memory": (4, "GiB")})]
    nd.compute_class()
    return nd


def alloc(i, prio, cpu, mem, devices=(), mbits=0, node="node-0", ports=()):
    """createAlloc; `mbits` is the bandwidth of the alloc's eth0 networks (task
    and group networks on one device add up in Flattened.Networks[0] and in
    NetworkIndex.UsedBandwidth alike); `ports` the (IP, value) ReservedPorts of
    its networks."""
    job = {LOW: "low", LOW2: "low2", HIGH: "high"}[prio]
    return Allocation(node_id=node, job_id=job, task_group="web", cpu_shares=cpu, memory_mb=mem,
                      disk_mb=0, priority=prio, devices=list(devices), net_mbits=mbits, ports=list(ports))


def ask_job(cpu, mem, device=None, mbits=0, ports=()):
    net = NetworkResource(mbits=mbits, reserved_ports=[v for _, v in ports],
                          port_labels=[lab for lab, _ in ports]) if (mbits or ports) else None
    return Job(id="preemptor", priority=100, task_groups=[TaskGroup(name="web", count=1, ephemeral_disk_mb=0, tasks=[
        Task(name="web", driver="exec", cpu=cpu, memory_mb=mem, network=net,
             devices=[device] if device else [])])])


CASES = {
    "one device instance per alloc": (
        [alloc(0, LOW, 500, 512, [(0, 1)]), alloc(1, LOW, 200, 512, [(0, 1)])],
        ask_job(1000, 512, RequestedDevice("nvidia/gpu/1080ti", 4)), {0, 1}),
    "multiple devices used": (
        [alloc(0, LOW, 500, 512, [(0, 4)]), alloc(1, LOW, 200, 512, [(2, 1)])],
        ask_job(1000, 512, RequestedDevice("nvidia/gpu/1080ti", 4)), {0}),
    "allocs across multiple devices that match": (
        [alloc(0, LOW, 500, 512, [(0, 2)]), alloc(1, HIGH, 200, 100, [(0, 1)]),
         alloc(2, LOW, 200, 256, [(1, 2)]), alloc(3, LOW, 100, 256, [(1, 2)]),
         alloc(4, LOW, 200, 512, [(2, 1)])],
        ask_job(1000, 512, RequestedDevice("gpu", 4)), {2, 3}),
    "lower/higher priority combinations": (
        [alloc(0, LOW, 500, 512, [(0, 2)]), alloc(1, LOW2, 200, 100, [(0, 2)]),
         alloc(2, LOW, 200, 256, [(1, 2)]), alloc(3, LOW, 100, 256, [(1, 2)]),
         alloc(4, LOW, 100, 256, [(1, 1)]), alloc(5, LOW, 200, 512, [(2, 1)])],
        ask_job(1000, 512, RequestedDevice("gpu", 4)), {2, 3}),
    "device preemption not possible": (
        [alloc(0, LOW, 500, 512, [(0, 4)]), alloc(1, LOW, 200, 512, [(2, 1)])],
        ask_job(1000, 512, RequestedDevice("gpu", 6)), None),
    # PreemptForNetwork (preemption.go:270-455) from BinPack's AssignNetwork failure
    "Combination of high/low priority allocs, without static ports": (
        [alloc(0, HIGH, 2800, 2256, mbits=150), alloc(1, LOW, 200, 256, mbits=200 + 300),
         alloc(2, LOW, 200, 256, mbits=300), alloc(3, LOW, 700, 256)],
        ask_job(1100, 1000, mbits=840), {1, 2, 3}),
    "preempt allocs with network devices": (
        [alloc(0, LOW, 2800, 2256), alloc(1, LOW, 200, 256, mbits=800)],
        ask_job(1100, 1000, mbits=840), {1}),
    "Preemption needed for all resources except network": (
        [alloc(0, HIGH, 2800, 2256, mbits=150), alloc(1, LOW, 200, 256, mbits=50),
         alloc(2, LOW, 200, 512), alloc(3, LOW, 700, 276)],
        ask_job(1000, 3000, mbits=50), {1, 2, 3}),
    "Only one low priority alloc needs to be preempted": (
        [alloc(0, HIGH, 1200, 2256, mbits=150), alloc(1, LOW, 200, 256, mbits=500),
         alloc(2, LOW, 200, 256, mbits=320)],
        ask_job(300, 500, mbits=320), {2}),
    "filter out superset allocs": (
        [alloc(0, HIGH, 1800, 2256, mbits=150), alloc(1, LOW, 1500, 256, mbits=100),
         alloc(2, LOW, 600, 256, mbits=300)],
        ask_job(1000, 256, mbits=50), {1}),
    # the task network asks static ports (AssignNetwork's ReservedPorts,
    # network.go:407-442; PreemptForNetwork's reserved-port step,
    # preemption.go:309-342). The reference node also carries mock.Node()'s
    # COMPAT Node.Reserved network (port 22 on 192.168.0.100), which is not
    # modelled; it changes no expected outcome below.
    "No preemption because existing allocs are not low priority": (
        [alloc(0, HIGH, 3200, 7256, mbits=50)],
        ask_job(2000, 256, mbits=1, ports=[("ssh", 22)]), None),
    "Preempting low priority allocs not enough to meet resource ask": (
        [alloc(0, LOW, 3200, 7256, mbits=50)],
        ask_job(4000, 8192, mbits=1, ports=[("ssh", 22)]), None),
    "preemption impossible - static port needed is used by higher priority alloc": (
        [alloc(0, HIGH, 1200, 2256, mbits=150), alloc(1, HIGH, 200, 256, mbits=600, ports=[("192.168.0.200", 88)])],
        ask_job(600, 1000, mbits=700, ports=[("db", 88)]), None),
    "one alloc meets static port need, another meets remaining mbits needed": (
        [alloc(0, HIGH, 1200, 2256, mbits=150), alloc(1, LOW, 200, 256, mbits=500, ports=[("192.168.0.200", 88)]),
         alloc(2, LOW, 200, 256, mbits=200)],
        ask_job(2700, 1000, mbits=800, ports=[("db", 88)]), {1, 2}),
    "alloc that meets static port need also meets other needs": (
        [alloc(0, HIGH, 1200, 2256, mbits=150), alloc(1, LOW, 200, 256, mbits=600, ports=[("192.168.0.200", 88)]),
         alloc(2, LOW, 200, 256, mbits=100)],
        ask_job(600, 1000, mbits=700, ports=[("db", 88)]), {1}),
}


def net_priority(prios):
    mx = float(max(prios))
    return mx + float(sum(prios)) / mx


@pytest.mark.parametrize("stack_cls", STACKS)
@pytest.mark.parametrize("case", list(CASES))
def test_preemption_kat(stack_cls, case):
    allocs, job, expected = CASES[case]
    node = preemption_node()
    st = stack_cls()
    st.SetState([node], allocs)
    st.SetJob(job)
    st.SetNodes([node])
    plain = st.SelectRaw(0)
    assert plain.row == -1                      # no fit without eviction
    r = st.SelectRaw(0, SelectOptions(preempt=True))
    if expected is None:
        assert r.row == -1
        return
    assert r.row == 0
    assert set(r.preempted) == expected
    # PreemptionScoringIterator: 1 / (1 + exp(0.0048 (netPriority - 2048))) appended last
    prios = [allocs[i].priority for i in r.preempted]
    want = 1.0 / (1.0 + math.exp(0.0048 * (net_priority(prios) - 2048.0)))
    assert abs(r.scores[-1] - want) <= 1e-12 * want


@pytest.mark.parametrize("stack_cls", STACKS)
def test_network_preemption_close_priority(stack_cls):
    """"ignore allocs with close enough priority for network devices": a job
    5 above the allocs finds no network candidate and the node is skipped."""
    node = preemption_node()
    allocs = [alloc(0, LOW, 2800, 2256), alloc(1, LOW, 200, 256, mbits=800)]
    job = ask_job(1100, 1000, mbits=840)
    job.priority = LOW + 5
    st = stack_cls()
    st.SetState([node], allocs)
    st.SetJob(job)
    st.SetNodes([node])
    r = st.SelectRaw(0, SelectOptions(preempt=True))
    assert r.row == -1 and r.nodes_exhausted == 0


@pytest.mark.parametrize("stack_cls", STACKS)
def test_network_preemption_existing_evictions(stack_cls):
    """"alloc from job that has existing evictions not chosen for preemption":
    the plan already preempts an alloc of the priority-40 job (here on a second
    node), the priority-30 alloc goes first and alone meets the bandwidth."""
    node = preemption_node()
    other = synth.mock_node("node-1")
    other.reserved_host_ports = []
    allocs = [alloc(0, HIGH, 1200, 2256, mbits=150), alloc(1, LOW, 200, 256, mbits=500),
              alloc(2, LOW2, 200, 256, mbits=300),
              alloc(3, LOW2, 3700, 256, mbits=300, node="node-1")]
    job = ask_job(300, 500, mbits=320)
    job.task_groups[0].count = 2
    st = stack_cls()
    st.SetState([node, other], allocs)
    st.SetJob(job)
    st.SetNodes([other])
    r1 = st.SelectRaw(0, SelectOptions(preempt=True))
    assert r1.row == 1 and r1.preempted == [3]
    st.Commit(0, r1.row, r1.preempted)
    st.SetNodes([node])
    r2 = st.SelectRaw(0, SelectOptions(preempt=True))
    assert r2.row == 0 and r2.preempted == [1]


@pytest.mark.parametrize("stack_cls", STACKS)
def test_group_port_preemption_frees_dynamic_ports(stack_cls):
    """AssignPorts failing on a task-group dynamic port ask with eviction
    (rank.go:273-300): PreemptForNetwork with an ask of 0 MBits keeps every
    alloc it collected (MeetsRequirements is false for 0 MBits), and only
    runs when the device's bandwidth is overcommitted; after the evictions
    the rebuilt index frees the dynamic ports."""
    nodes = [synth.mock_node("n%d" % i) for i in range(4)]
    for nd in nodes:
        nd.compute_class()
    allocs = []
    for i, nd in enumerate(nodes):
        allocs.append(Allocation(node_id=nd.id, job_id="batch-%d" % i, task_group="t", cpu_shares=600,
                                 memory_mb=256, priority=20, dyn_ports=12001, net_mbits=700))
        allocs.append(Allocation(node_id=nd.id, job_id="svc-%d" % i, task_group="t", cpu_shares=600,
                                 memory_mb=256, priority=30, net_mbits=400 if i % 2 else 200))
    job = synth.mock_job(count=3)
    job.priority = 70
    st = stack_cls(config=SchedulerConfig(preempt_service=True))
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes(list(range(len(nodes))))
    r = st.SelectRaw(0, SelectOptions(preempt=True))
    # nodes 1, 3 are overcommitted (1100 > 1000 MBits): the priority-20 alloc
    # goes first and is enough; nodes 0, 2 are skipped
    assert (r.row, r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted) == (1, 4, 0, 0)
    assert r.preempted == [2]


@pytest.mark.parametrize("stack_cls", STACKS)
def test_static_port_holder_on_the_address_is_preempted(stack_cls):
    """A task static port held on the node's address by a low-priority alloc:
    AssignNetwork fails, PreemptForNetwork takes the port holder first
    (usedPortToAlloc), which also frees enough bandwidth; the retried offer
    gets the port."""
    node = preemption_node()
    allocs = [alloc(0, HIGH, 1200, 2256, mbits=150),
              alloc(1, LOW, 200, 256, mbits=600, ports=[("192.168.0.100", 88)]),
              alloc(2, LOW, 200, 256, mbits=50)]
    job = ask_job(600, 1000, mbits=100, ports=[("db", 88)])
    st = stack_cls()
    st.SetState([node], allocs)
    st.SetJob(job)
    st.SetNodes([node])
    assert st.SelectRaw(0).row == -1          # reserved port collision db=88
    r = st.SelectRaw(0, SelectOptions(preempt=True))
    assert r.row == 0 and r.preempted == [1]


@pytest.mark.parametrize("stack_cls", STACKS)
def test_static_port_held_by_a_close_priority_alloc(stack_cls):
    """filteredReservedPorts: the port is held by an alloc too close in
    priority; no preemption even though another candidate would free
    bandwidth."""
    node = preemption_node()
    allocs = [alloc(0, LOW, 1200, 2256, mbits=300),
              alloc(1, HIGH, 200, 256, mbits=100, ports=[("192.168.0.100", 88)])]
    job = ask_job(600, 1000, mbits=100, ports=[("db", 88)])
    st = stack_cls()
    st.SetState([node], allocs)
    st.SetJob(job)
    st.SetNodes([node])
    assert st.SelectRaw(0, SelectOptions(preempt=True)).row == -1


@pytest.mark.parametrize("stack_cls", STACKS)
def test_group_static_port_preemption(stack_cls):
    """Task-group static ports (AssignPorts, rank.go:265-300): the holder of the
    port on the host network's address is preempted; a node whose port is a
    node reservation stays skipped."""
    nodes = [synth.mock_node("n%d" % i) for i in range(3)]
    nodes[2].reserved_host_ports = [22, 8080]
    for nd in nodes:
        nd.compute_class()
    allocs = [Allocation(node_id="n0", job_id="svc", task_group="t", cpu_shares=3000, memory_mb=512,
                         priority=80, ports=[("192.168.0.100", 8080)], net_mbits=10),
              Allocation(node_id="n1", job_id="batch", task_group="t", cpu_shares=500, memory_mb=512,
                         priority=20, ports=[("192.168.0.100", 8080)], net_mbits=10),
              Allocation(node_id="n1", job_id="batch2", task_group="t", cpu_shares=500, memory_mb=512,
                         priority=20, net_mbits=10)]
    job = synth.mock_job(count=2)
    job.priority = 70
    job.task_groups[0].network = NetworkResource(mode="host", dynamic_ports=1, reserved_ports=[8080],
                                                 port_labels=["http"])
    st = stack_cls(config=SchedulerConfig(preempt_service=True))
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes([0, 1, 2])
    assert st.SelectRaw(0).row == -1
    r = st.SelectRaw(0, SelectOptions(preempt=True))
    assert (r.row, r.preempted, r.nodes_evaluated) == (1, [1], 3)


@pytest.mark.parametrize("stack_cls", STACKS)
def test_preemption_commit_frees_resources(stack_cls):
    """Plan.AppendPreemptedAlloc removes the victims from ProposedAllocs
    (context.go:134-138): after the preempting placement commits, the freed
    instances are gone to the new alloc and a second identical ask needs
    another eviction round."""
    allocs, job, _ = CASES["one device instance per alloc"]
    node = preemption_node()
    st = stack_cls()
    st.SetState([node], allocs)
    st.SetJob(job)
    st.SetNodes([node])
    r = st.SelectRaw(0, SelectOptions(preempt=True))
    st.Commit(0, r.row, r.preempted)
    again = st.SelectRaw(0, SelectOptions(preempt=True))
    assert again.row == -1                      # 1080ti fully held by our own alloc


@pytest.mark.parametrize("stack_cls", STACKS)
def test_max_parallel_penalty(stack_cls):
    """scoreForTaskGroup adds 50 x (preempted + 1 - maxParallel) once a job's
    preemptions in the plan reach its migrate max_parallel
    (preemption.go:633-642): the penalised alloc is passed over."""
    node = preemption_node()
    allocs = [Allocation(node_id="node-0", job_id="a", task_group="web", cpu_shares=1900, memory_mb=256,
                         priority=LOW, max_parallel=1),
              Allocation(node_id="node-0", job_id="b", task_group="web", cpu_shares=1950, memory_mb=256,
                         priority=LOW),
              Allocation(node_id="node-0", job_id="a", task_group="web", cpu_shares=10, memory_mb=10,
                         priority=LOW, max_parallel=1)]
    other = synth.mock_node("node-1")
    other.reserved_host_ports = []
    job = ask_job(1900, 256)
    job.task_groups[0].count = 2
    st = stack_cls()
    st.SetState([node, other], allocs + [Allocation(node_id="node-1", job_id="a", task_group="web",
                                                    cpu_shares=3000, memory_mb=64, priority=LOW,
                                                    max_parallel=1)])
    st.SetJob(job)
    st.SetNodes([other])
    r1 = st.SelectRaw(0, SelectOptions(preempt=True))
    assert r1.row == 1 and r1.preempted == [3]          # job "a" now has one preemption in the plan
    st.Commit(0, r1.row, r1.preempted)
    st.SetNodes([node])
    r2 = st.SelectRaw(0, SelectOptions(preempt=True))
    assert r2.row == 0 and r2.preempted == [1]          # alloc 0 (closer) carries the +50 penalty


# ---- GPU parity: count loop with preemption fallback (C5) ---------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("n,count,seed", [(400, 300, 1), (2000, 1500, 2)])
def test_c5_preemption_count_loop(n, count, seed):
    nodes, allocs = synth.cluster_c5(n, seed=seed)
    job = synth.job_c5(count)
    perm = synth.shuffle(len(nodes), seed + 20)
    cfg = SchedulerConfig(preempt_service=True)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm, config=cfg)
    _, _, re = run_place(_engine, nodes, allocs, job, perm, config=cfg)
    assert any(x.preempted for x in ro)                 # the workload exercises eviction
    assert_same_placements(re, ro)
    assert [sorted(x.preempted) for x in re] == [sorted(x.preempted) for x in ro]
    assert [x.device_offers for x in re] == [x.device_offers for x in ro]


def _system_place(cls, nodes, allocs, job, cfg):
    st = cls(config=cfg)
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes(list(range(len(nodes))))
    return st.SystemPlace(0)


@pytest.mark.parametrize("max_parallel", [False, True])
def test_system_preemption_oracle_places_more(max_parallel):
    """SystemStack BinPack evicts when preemption is enabled (stack.go:267-278):
    with it, nodes full of priority-20 GPU work take the system job."""
    from oracle.oracle import OracleSystemStack
    nodes, allocs = synth.cluster_c5(300, seed=8)
    if not max_parallel:
        for a in allocs:
            a.max_parallel = 0
    job = synth.job_c5(1)
    job.type = 2
    _, s0, p0 = _system_place(OracleSystemStack, nodes, allocs, job, SchedulerConfig())
    _, s1, p1 = _system_place(OracleSystemStack, nodes, allocs, job, SchedulerConfig(preempt_system=True))
    assert p1 > p0


@pytest.mark.gpu
@pytest.mark.parametrize("max_parallel", [False, True])
def test_system_preemption_parity(max_parallel):
    from nomad_amd.stack import SystemStack
    from oracle.oracle import OracleSystemStack
    nodes, allocs = synth.cluster_c5(3000, seed=9)
    if not max_parallel:
        for a in allocs:
            a.max_parallel = 0
    job = synth.job_c5(1)
    job.type = 2
    cfg = SchedulerConfig(preempt_system=True)
    so, to, po = _system_place(OracleSystemStack, nodes, allocs, job, cfg)
    se, te, pe = _system_place(SystemStack, nodes, allocs, job, cfg)
    assert po == pe and (to == te).all()
    m = to == 0
    assert (so[m] == se[m]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("preempt", [False, True])
def test_c5_sparse_parallel_count_loop(preempt):
    """A saturated cluster (options sparse): the engine's count loop evaluates
    each Select in parallel and resolves the window on the device."""
    nodes, allocs = synth.cluster_c5(5000, seed=3, busy=0.99)
    job = synth.job_c5(120)
    perm = synth.shuffle(len(nodes), 31)
    cfg = SchedulerConfig(preempt_service=preempt)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, job, perm, config=cfg)
    _, _, re = run_place(_engine, nodes, allocs, job, perm, config=cfg)
    assert_same_placements(re, ro)
    assert [sorted(x.preempted) for x in re] == [sorted(x.preempted) for x in ro]


@pytest.mark.parametrize("stack_cls", STACKS)
def test_preempt_skips_nodes_without_dynamic_ports(stack_cls):
    """BinPack with evict on a task-group port ask that a node cannot meet:
    PreemptForNetwork (preemption.go:270-455) finds nothing to evict while the
    node's bandwidth is not overcommitted, and the node is skipped
    (rank.go:265-272) -- neither filtered nor exhausted."""
    nodes = [synth.mock_node("n%d" % i) for i in range(6)]
    for nd in nodes:
        nd.compute_class()
    allocs = []
    for i, nd in enumerate(nodes):
        # low-priority work fills cpu everywhere; nodes 0, 2, 4 also hold every dynamic port
        allocs.append(Allocation(node_id=nd.id, job_id="batch-%d" % i, task_group="t", cpu_shares=3800,
                                 memory_mb=256, priority=20, dyn_ports=12001 if i % 2 == 0 else 0))
    job = synth.mock_job(count=3)
    job.priority = 70
    st = stack_cls(config=SchedulerConfig(preempt_service=True))
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes(list(range(len(nodes))))
    r = st.SelectRaw(0, SelectOptions(preempt=True))
    # nodes 0, 2, 4 are skipped; 1, 3, 5 evict their batch alloc (limit 3); the first wins the tie
    assert (r.row, r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted) == (1, 6, 0, 0)
    assert r.preempted == [1]


def two_nic_node():
    """preemption_test.go:408's node: preemption_node() with a second host
    network device, eth0 192.168.0.100/32 and eth1 192.168.1.100/32 at 1000
    MBits each."""
    nd = preemption_node()
    nd.networks = [NetworkResource(mode="host", device="eth0", cidr="192.168.0.100/32", mbits=1000),
                   NetworkResource(mode="host", device="eth1", cidr="192.168.1.100/32", mbits=1000)]
    nd.compute_class()
    return nd


def on(dev, a):
    a.net_device = dev
    return a


@pytest.mark.parametrize("stack_cls", STACKS)
def test_preempt_only_from_device_with_unused_reserved_port(stack_cls):
    """"preempt only from device that has allocation with unused reserved port"
    (preemption_test.go:408-496): bandwidth is kept per device
    (NetworkIndex.UsedBandwidth[device], network.go:196-230), AssignNetwork
    walks the node's two devices (yieldIP, network.go:294-315, 407-482) and
    finds neither with 700 MBits free; PreemptForNetwork groups the candidates
    by device (preemption.go:292-331): only eth0 holds a low-priority one, the
    high-priority holder of port 88 sits on eth1, so the low-priority eth0
    alloc is preempted and the retried offer lands on eth0."""
    node = two_nic_node()
    allocs = [on("eth0", alloc(0, HIGH, 1200, 2256, mbits=150)),
              on("eth1", alloc(1, HIGH, 200, 256, mbits=600, ports=[("192.168.0.200", 88)])),
              on("eth0", alloc(2, LOW, 200, 256, mbits=600))]
    job = ask_job(600, 1000, mbits=700, ports=[("db", 88)])
    st = stack_cls()
    st.SetState([node], allocs)
    st.SetJob(job)
    st.SetNodes([node])
    plain = st.SelectRaw(0)
    assert plain.row == -1 and plain.nodes_exhausted == 1
    r = st.SelectRaw(0, SelectOptions(preempt=True))
    assert r.row == 0 and set(r.preempted) == {2}
    want = 1.0 / (1.0 + math.exp(0.0048 * (net_priority([LOW]) - 2048.0)))
    assert abs(r.scores[-1] - want) <= 1e-12 * want


@pytest.mark.parametrize("stack_cls", STACKS)
def test_candidates_on_two_devices_are_refused(stack_cls):
    """PreemptForNetwork ranges over its deviceToAllocs map
    (preemption.go:335-408): with preemptible candidates on both devices the
    reference's answer depends on Go's map order, so both sides refuse
    (PE_EUNSUPPORTED / oracle Unsupported) and the caller's chain answers; with
    the eth1 candidate raised to a close priority only eth0 has candidates and
    the answer is the reference's."""
    node = two_nic_node()
    job = ask_job(600, 1000, mbits=700)
    for prio1, refused in ((LOW, True), (HIGH, False)):
        allocs = [on("eth0", alloc(0, HIGH, 1200, 2256, mbits=150)),
                  on("eth1", alloc(1, prio1, 200, 256, mbits=600)),
                  on("eth0", alloc(2, LOW, 200, 256, mbits=600))]
        st = stack_cls()
        st.SetState([node], allocs)
        st.SetJob(job)
        st.SetNodes([node])
        assert st.SelectRaw(0).row == -1
        if refused:
            with pytest.raises(Exception, match="(?i)unsupported|network device"):
                st.SelectRaw(0, SelectOptions(preempt=True))
        else:
            r = st.SelectRaw(0, SelectOptions(preempt=True))
            assert r.row == 0 and r.preempted == [2]


@pytest.mark.parametrize("stack_cls", STACKS)
def test_alloc_on_a_device_the_node_lacks(stack_cls):
    """An alloc whose network names a device the node has no network for
    holds bandwidth on that device only (UsedBandwidth[device]): the node's
    eth0 keeps its 1000 MBits and the 840-MBit ask places without eviction.
    With the alloc on eth0 the network is short and PreemptForNetwork picks it."""
    node = preemption_node()
    job = ask_job(1100, 1000, mbits=840)
    for dev in ("eth1", "eth0"):
        allocs = [alloc(0, LOW, 2000, 2256), on(dev, alloc(1, LOW, 200, 256, mbits=800))]
        st = stack_cls()
        st.SetState([node], allocs)
        st.SetJob(job)
        st.SetNodes([node])
        plain = st.SelectRaw(0)
        if dev == "eth1":
            assert plain.row == 0 and plain.preempted == []
        else:
            assert plain.row == -1
            r = st.SelectRaw(0, SelectOptions(preempt=True))
            assert r.row == 0 and r.preempted == [1]
