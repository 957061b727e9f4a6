"""Synthetic snapshots and plans for the plan applier (tests and bench).

`mock_node` / `mock_alloc` / `nvidia_node` restate the reference fixtures
mock.Node(), mock.Alloc(), mock.NvidiaNode() (nomad/mock/mock.go:14-152,
1277-1345) in the plan applier's view. `random_case` draws seeded edge-heavy
snapshots + plans (cores, port specs, invalid ports, devices, terminal /
removed / updated allocs, missing / down / ineligible nodes, nodes past the
LDS key budget). `system_plan` builds the bench workload: a system-job plan
placing one alloc on every node of a large cluster (SURVEY.md §8d C4 shape).
"""
from __future__ import annotations

import random
import uuid
from typing import List, Tuple

from .plan import (AllocDevice, AllocNetwork, NodeDevice, NodeDeviceResource, NodeNetworkAddress, Plan, PlanAlloc,
                   PlanNode, Port)


def _uuid(rng: random.Random) -> str:
    return str(uuid.UUID(int=rng.getrandbits(128), version=4))


def mock_node(node_id: str) -> PlanNode:
    """mock.Node(): NodeResources 4000/8192/100 GiB, ReservedResources 100/256/4 GiB
    with ReservedHostPorts "22", one host network eth0 (CIDR, no IP) and the
    NodeNetworks address 192.168.0.100."""
    return PlanNode(id=node_id, cpu_shares=4000, memory_mb=8192, disk_mb=100 * 1024, reserved_cpu=100,
                    reserved_memory_mb=256, reserved_disk_mb=4 * 1024, networks=[("eth0", "")],
                    addresses=[NodeNetworkAddress(address="192.168.0.100")], reserved_host_ports="22")


def nvidia_node(node_id: str, instance_ids: List[str]) -> PlanNode:
    n = mock_node(node_id)
    n.devices = [NodeDeviceResource("nvidia", "gpu", "1080ti", [NodeDevice(i, True) for i in instance_ids])]
    return n


def mock_alloc(alloc_id: str, node_id: str = "12345678-abcd-efab-cdef-123456789abc") -> PlanAlloc:
    """mock.Alloc(): task "web" 500 MHz / 256 MB, disk 150, network on
    192.168.0.100 with reserved port 5000 and dynamic port 9876."""
    return PlanAlloc(id=alloc_id, node_id=node_id, cpu_shares=500, memory_mb=256, disk_mb=150,
                     task_networks={"web": [AllocNetwork(ip="192.168.0.100", device="eth0", mbits=50,
                                                         reserved_ports=[5000], dynamic_ports=[9876])]})


def full_node_alloc(alloc_id: str, node: PlanNode) -> PlanAlloc:
    """structs.NodeResourcesToAllocatedResources(node.NodeResources) (testing.go:14-34)."""
    return PlanAlloc(id=alloc_id, node_id=node.id, cpu_shares=node.cpu_shares, memory_mb=node.memory_mb,
                     disk_mb=node.disk_mb)


_SPECS = ["", "22", "22,80", "80-82", "8000-8002,22", "bad", "70000", "22,", "5-3", " 9876 ", "1-2-3", "65535-65540"]
_IPS = ["192.168.0.100", "10.0.0.1", ""]


def random_case(seed: int, n_nodes: int = 24, max_allocs: int = 4, big_keys: bool = False
                ) -> Tuple[List[PlanNode], List[PlanAlloc], Plan]:
    rng = random.Random(seed)
    nodes: List[PlanNode] = []
    for _ in range(n_nodes):
        nid = _uuid(rng)
        n = PlanNode(id=nid, cpu_shares=rng.choice([2000, 4000, 8000]), memory_mb=rng.choice([4096, 8192]),
                     disk_mb=rng.choice([20000, 100000]))
        if rng.random() < 0.8:
            n.reserved_cpu, n.reserved_memory_mb, n.reserved_disk_mb = 100, 256, 4096
        n.status = "ready" if rng.random() < 0.9 else rng.choice(["init", "down"])
        n.scheduling_eligibility = "eligible" if rng.random() < 0.9 else "ineligible"
        if rng.random() < 0.4:
            ncores = 600 if big_keys and rng.random() < 0.5 else rng.choice([4, 8])
            n.reservable_cores = list(range(ncores))
            n.reserved_cores = [0] if rng.random() < 0.5 else []
        n.networks = [("eth0", rng.choice(_IPS))] + ([("", "1.1.1.1")] if rng.random() < 0.2 else [])
        for _ in range(rng.randint(0, 2)):
            n.addresses.append(NodeNetworkAddress(address=rng.choice(_IPS[:2]), reserved_ports=rng.choice(_SPECS)))
        n.reserved_host_ports = rng.choice(_SPECS)
        if rng.random() < 0.5:
            for g in range(rng.randint(1, 2)):
                inst = [NodeDevice(_uuid(rng), rng.random() < 0.8) for _ in range(rng.randint(1, 4))]
                n.devices.append(NodeDeviceResource("nvidia", "gpu", rng.choice(["a100", "1080ti"]), inst))
        nodes.append(n)

    def rand_alloc(node: PlanNode) -> PlanAlloc:
        a = PlanAlloc(id=_uuid(rng), node_id=node.id, cpu_shares=rng.choice([100, 500, 1500, 3000]),
                      memory_mb=rng.choice([128, 256, 2048, 6000]), disk_mb=rng.choice([150, 5000, 50000]))
        r = rng.random()
        if r < 0.1:
            a.desired_status = rng.choice(["stop", "evict"])
        elif r < 0.15:
            a.client_status = rng.choice(["complete", "failed", "lost"])
        if node.reservable_cores and rng.random() < 0.5:
            pool = node.reservable_cores + [999]
            a.reserved_cores = rng.sample(pool, min(len(pool), rng.randint(1, 3)))
        pr = rng.random()
        port = lambda: rng.choice([22, 80, 5000, 9876, 8001, rng.randint(20000, 32000), -1, 70000]) \
            if rng.random() < 0.95 else rng.choice([-5, 65536])
        if pr < 0.35:
            a.shared_ports = [Port(port(), rng.choice(_IPS)) for _ in range(rng.randint(1, 3))]
        elif pr < 0.7:
            a.task_networks = {"web": [AllocNetwork(ip=rng.choice(_IPS), reserved_ports=[port()],
                                                    dynamic_ports=[port()])]}
            if rng.random() < 0.3:
                a.shared_networks = [AllocNetwork(ip=rng.choice(_IPS), dynamic_ports=[port()])]
        if node.devices and rng.random() < 0.6:
            g = rng.choice(node.devices)
            ids = [i.id for i in g.instances]
            pick = rng.sample(ids, min(len(ids), rng.randint(1, 2)))
            if rng.random() < 0.1:
                pick.append(_uuid(rng))   # unknown instance: ignored by the accounter
            a.devices = [AllocDevice(g.vendor, g.type, g.name if rng.random() < 0.9 else "other", pick)]
        return a

    allocs: List[PlanAlloc] = []
    for n in nodes:
        for _ in range(rng.randint(0, max_allocs)):
            allocs.append(rand_alloc(n))
    by_node = {}
    for a in allocs:
        by_node.setdefault(a.node_id, []).append(a)

    plan = Plan(all_at_once=rng.random() < 0.1)
    for n in nodes:
        r = rng.random()
        existing = by_node.get(n.id, [])
        if r < 0.15 and existing:                     # evict-only
            plan.node_update[n.id] = [rng.choice(existing)]
            continue
        if r < 0.25:
            continue
        placed = [rand_alloc(n) for _ in range(rng.randint(1, 3))]
        if existing and rng.random() < 0.3:           # in-place update of an existing alloc
            old = rng.choice(existing)
            upd = rand_alloc(n)
            upd.id = old.id
            placed.append(upd)
        plan.node_allocation[n.id] = placed
        if existing and rng.random() < 0.3:
            plan.node_update[n.id] = [rng.choice(existing)]
        if existing and rng.random() < 0.3:
            plan.node_preemptions[n.id] = [rng.choice(existing)]
    if rng.random() < 0.5:
        ghost = _uuid(rng)
        plan.node_allocation[ghost] = [rand_alloc(PlanNode(id=ghost))]
    return nodes, allocs, plan


def system_plan(n_nodes: int, seed: int = 42) -> Tuple[List[PlanNode], List[PlanAlloc], Plan]:
    """Bench workload: n_nodes mock-like nodes (4-64 reservable cores, reserved
    host port 22, 0-3 existing allocs with ports, 40% with 4-8 GPU instances);
    the plan places one system alloc (500 MHz / 256 MB, one dynamic port, 5% on
    a taken port, 5% over capacity) on every node."""
    rng = random.Random(seed)
    nodes, allocs = [], []
    plan = Plan()
    for i in range(n_nodes):
        nid = "%08x-0000-4000-8000-%012x" % (i, i)
        ip = "10.%d.%d.%d" % (i >> 16 & 255, i >> 8 & 255, i & 255)
        n = PlanNode(id=nid, cpu_shares=rng.choice([4000, 8000, 16000, 32000]),
                     memory_mb=rng.choice([8192, 16384, 65536]), disk_mb=rng.choice([102400, 204800]),
                     reserved_cpu=100, reserved_memory_mb=256, reserved_disk_mb=4096,
                     networks=[("eth0", "")], addresses=[NodeNetworkAddress(address=ip)], reserved_host_ports="22")
        n.reservable_cores = list(range(rng.choice([4, 8, 16, 32, 64])))
        if rng.random() < 0.4:
            n.devices = [NodeDeviceResource("nvidia", "gpu", "a100",
                                            [NodeDevice("%s-gpu%d" % (nid, k)) for k in range(rng.choice([4, 8]))])]
        nodes.append(n)
        used_ports = []
        for k in range(rng.randint(0, 3)):
            p = 20000 + rng.randrange(12000)
            used_ports.append(p)
            a = PlanAlloc(id="%s-a%d" % (nid, k), node_id=nid, cpu_shares=rng.choice([250, 500, 1000]),
                          memory_mb=rng.choice([128, 256, 1024]), disk_mb=150, shared_ports=[Port(p, ip)])
            if n.devices and k == 0:
                a.devices = [AllocDevice("nvidia", "gpu", "a100", [n.devices[0].instances[0].id])]
            if rng.random() < 0.3:
                a.reserved_cores = [k]
            allocs.append(a)
        r = rng.random()
        port = rng.choice(used_ports) if (r < 0.05 and used_ports) else 20000 + rng.randrange(12000)
        cpu = n.cpu_shares if 0.05 <= r < 0.10 else 500
        plan.node_allocation[nid] = [PlanAlloc(id="%s-sys" % nid, node_id=nid, cpu_shares=cpu, memory_mb=256,
                                               disk_mb=150, shared_ports=[Port(port, ip)])]
    return nodes, allocs, plan
