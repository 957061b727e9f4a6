"""Seeded synthetic clusters and jobs for the BASELINE.json configs.

  C1  100 mock.Node() clones + mock.Job() (count 10)          nomad/mock/mock.go:14-119, 232-337
  C2  10k heterogeneous nodes, count=1000 binpack service job  
  C3  10k nodes / 3 DCs, semver + regexp constraints, affinity, spread
  C4  system job (mock.SystemJob, mock.go:1141-1201) on a large cluster
  C5  device asks (nvidia/gpu count 2, memory constraint) with preemption of
      priority-20 background allocs (mock.NvidiaNode, mock.go:131-158)

Node IDs are deterministic UUIDs from a seeded generator so the memdb order
(ascending ID, nomad/state/schema.go:109-115) is fixed. `shuffle` stands in
for shuffleNodes (scheduler/util.go:366-372): Fisher-Yates driven by a seeded
PCG64 instead of Go's math/rand (whose stream cannot be reproduced without a
Go toolchain; the permutation is an input of the engine).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from .structs import (Affinity, Allocation, Constraint, DeviceGroup, DriverInfo, Job, NetworkResource, Node,
                      RequestedDevice, Spread, SpreadTarget, Task, TaskGroup)


def uuids(n: int, seed: int) -> List[str]:
    rng = np.random.Generator(np.random.PCG64(seed))
    raw = rng.integers(0, 2 ** 63, size=(n, 2), dtype=np.int64).astype(np.uint64)
    out = []
    for a, b in raw:
        h = "%016x%016x" % (int(a), int(b))
        out.append("%s-%s-%s-%s-%s" % (h[0:8], h[8:12], h[12:16], h[16:20], h[20:32]))
    return out


def shuffle(n: int, seed: int) -> np.ndarray:
    """Fisher-Yates: for i = n-1..1, j = Intn(i+1), swap (util.go:366-372)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    perm = np.arange(n, dtype=np.uint32)
    if n > 1:
        js = [int(rng.integers(0, i + 1)) for i in range(n - 1, 0, -1)]
        for i, j in zip(range(n - 1, 0, -1), js):
            perm[i], perm[j] = perm[j], perm[i]
    return perm


def mock_node(node_id: str) -> Node:
    """mock.Node() (nomad/mock/mock.go:14-119)."""
    n = Node(
        id=node_id, name="foobar", datacenter="dc1", node_class="linux-medium-pci",
        attributes={"kernel.name": "linux", "arch": "x86", "nomad.version": "0.5.0",
                    "driver.exec": "1", "driver.mock_driver": "1"},
        meta={"pci-dss": "true", "database": "mysql", "version": "5.6"},
        drivers={"exec": DriverInfo(True, True), "mock_driver": DriverInfo(True, True)},
        cpu_shares=4000, memory_mb=8192, disk_mb=100 * 1024,
        reserved_cpu=100, reserved_memory_mb=256, reserved_disk_mb=4 * 1024,
        networks=[NetworkResource(mode="host", device="eth0", cidr="192.168.0.100/32", mbits=1000)],
        host_network_aliases=["default"], reserved_host_ports=[22],
    )
    n.compute_class()
    return n


def mock_job(job_id: str = "mock-service-0", count: int = 10) -> Job:
    """mock.Job() (nomad/mock/mock.go:232-337), canonicalized."""
    return Job(
        id=job_id, priority=50, datacenters=["dc1"],
        constraints=[Constraint("${attr.kernel.name}", "linux", "=")],
        task_groups=[TaskGroup(
            name="web", count=count, ephemeral_disk_mb=150,
            network=NetworkResource(mode="host", dynamic_ports=2, host_network="default"),
            tasks=[Task(name="web", driver="exec", cpu=500, memory_mb=256)])],
    )


def mock_system_job(job_id: str = "mock-system-0") -> Job:
    """mock.SystemJob() (nomad/mock/mock.go:1141-1201): task network 50 MBits + 1 dyn port."""
    return Job(
        id=job_id, type=2, priority=100, datacenters=["dc1"],
        constraints=[Constraint("${attr.kernel.name}", "linux", "=")],
        task_groups=[TaskGroup(
            name="web", count=1, ephemeral_disk_mb=300,
            tasks=[Task(name="web", driver="exec", cpu=500, memory_mb=256,
                        network=NetworkResource(mbits=50, dynamic_ports=1))])],
    )


def cluster_c1(n: int = 100, seed: int = 42) -> Tuple[List[Node], List[Allocation]]:
    ids = sorted(uuids(n, seed))
    return [mock_node(i) for i in ids], []


CPU_CHOICES = np.array([4000, 8000, 16000, 32000, 64000])
MEM_CHOICES = np.array([8192, 16384, 32768, 65536, 131072])


def cluster_c2(n: int = 10000, seed: int = 42, other_allocs: bool = True):
    """10k heterogeneous nodes, 1 DC, ~8 computed classes, 0-3 foreign allocs per node."""
    rng = np.random.Generator(np.random.PCG64(seed))
    ids = sorted(uuids(n, seed))
    nodes, allocs = [], []
    for k, nid in enumerate(ids):
        cls = int(rng.integers(0, 8))
        cpu = int(CPU_CHOICES[rng.integers(0, 5)])
        mem = int(MEM_CHOICES[rng.integers(0, 5)])
        disk = int(rng.integers(100, 501)) * 1024
        nd = mock_node(nid)
        nd.name = "node-%05d" % k
        nd.node_class = "class-%d" % cls
        nd.attributes["cpu.arch"] = "amd64" if cls % 2 == 0 else "arm64"
        nd.cpu_shares, nd.memory_mb, nd.disk_mb = cpu, mem, disk
        nd.compute_class()
        nodes.append(nd)
        if other_allocs:
            free_c, free_m = cpu - 100, mem - 256
            for a in range(int(rng.integers(0, 4))):
                c = int(rng.integers(250, 2001))
                m = int(rng.integers(128, 4097))
                if c <= free_c and m <= free_m:
                    free_c -= c
                    free_m -= m
                    allocs.append(Allocation(node_id=nid, job_id="other-%d" % (k % 97), task_group="tg",
                                             cpu_shares=c, memory_mb=m, disk_mb=300, priority=50))
    return nodes, allocs


def job_c2(count: int = 1000) -> Job:
    return Job(
        id="svc-c2", priority=50, datacenters=["dc1"],
        constraints=[Constraint("${attr.kernel.name}", "linux", "=")],
        task_groups=[TaskGroup(name="web", count=count, ephemeral_disk_mb=150,
                               tasks=[Task(name="web", driver="exec", cpu=500, memory_mb=256)])],
    )


def cluster_c3(n: int = 10000, seed: int = 7):
    """3 DCs 50/30/20 %, linux 95 %, os.version mix, meta.rack r00-r99, node_class c0-c7."""
    rng = np.random.Generator(np.random.PCG64(seed))
    ids = sorted(uuids(n, seed))
    versions = ["4.19.0", "5.4.0", "5.10.12", "6.1.0-rc1"]
    nodes = []
    for k, nid in enumerate(ids):
        u = rng.random()
        dc = "dc1" if u < 0.5 else ("dc2" if u < 0.8 else "dc3")
        nd = mock_node(nid)
        nd.name = "node-%05d" % k
        nd.datacenter = dc
        nd.attributes["kernel.name"] = "linux" if rng.random() < 0.95 else "windows"
        nd.attributes["os.version"] = versions[int(rng.integers(0, 4))]
        nd.meta["rack"] = "r%02d" % int(rng.integers(0, 100))
        nd.node_class = "c%d" % int(rng.integers(0, 8))
        nd.cpu_shares = int(CPU_CHOICES[rng.integers(0, 3)])
        nd.memory_mb = int(MEM_CHOICES[rng.integers(0, 3)])
        nd.compute_class()
        nodes.append(nd)
    return nodes, []


def job_c3(count: int = 1000) -> Job:
    return Job(
        id="svc-c3", priority=50, datacenters=["dc1", "dc2", "dc3"],
        constraints=[Constraint("${attr.kernel.name}", "linux", "="),
                     Constraint("${attr.os.version}", ">= 5.4.0", "semver"),
                     Constraint("${meta.rack}", "^r[0-4]", "regexp")],
        affinities=[Affinity("${node.class}", "c3", "=", 50)],
        spreads=[Spread("${node.datacenter}", 100, [SpreadTarget("dc1", 50), SpreadTarget("dc2", 30)])],
        task_groups=[TaskGroup(name="web", count=count, ephemeral_disk_mb=150,
                               tasks=[Task(name="web", driver="exec", cpu=250, memory_mb=128)])],
    )


def cluster_c4(n: int = 100000, seed: int = 11):
    """System-job cluster: ~10 % windows (constraint-filtered), ~5 % pre-filled (exhausted)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    ids = sorted(uuids(n, seed))
    nodes, allocs = [], []
    for k, nid in enumerate(ids):
        nd = mock_node(nid)
        nd.name = "node-%06d" % k
        if rng.random() < 0.10:
            nd.attributes["kernel.name"] = "windows"
        nd.cpu_shares = int(CPU_CHOICES[rng.integers(0, 3)])
        nd.compute_class()
        nodes.append(nd)
        if rng.random() < 0.05:
            allocs.append(Allocation(node_id=nid, job_id="filler", task_group="tg",
                                     cpu_shares=nd.cpu_shares - 100 - 100, memory_mb=1024,
                                     disk_mb=300, priority=50))
    return nodes, allocs


GPU_MODELS = {   # name -> device attributes (mock.NvidiaNode attribute set)
    "a100": {"memory": (80, "GiB"), "cuda_cores": 6912, "graphics_clock": (1410, "MHz"),
             "memory_bandwidth": (2039, "GB/s")},
    "h100": {"memory": (80, "GiB"), "cuda_cores": 16896, "graphics_clock": (1755, "MHz"),
             "memory_bandwidth": (3350, "GB/s")},
    "1080ti": {"memory": (11, "GiB"), "cuda_cores": 3584, "graphics_clock": (1480, "MHz"),
               "memory_bandwidth": (11, "GB/s")},
}


def nvidia_node(node_id: str, model: str = "1080ti", healthy: int = 2) -> Node:
    """mock.NvidiaNode() (mock.go:131-158) with a chosen model / instance count."""
    nd = mock_node(node_id)
    nd.devices = [DeviceGroup("nvidia", "gpu", model, healthy, dict(GPU_MODELS[model]))]
    nd.compute_class()
    return nd


def cluster_c5(n: int = 50000, seed: int = 5, busy: float = 0.0):
    """60 % of the nodes carry one nvidia/gpu group (a100 / h100 / 1080ti, 4 or 8
    healthy instances); priority-20 background allocs hold 0..all instances
    (all of them on a `busy` fraction of the GPU nodes, so that a count=1000
    ask must preempt)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    ids = sorted(uuids(n, seed))
    models = ["a100", "h100", "1080ti"]
    nodes, allocs = [], []
    for k, nid in enumerate(ids):
        nd = mock_node(nid)
        nd.name = "node-%05d" % k
        nd.cpu_shares = int(CPU_CHOICES[rng.integers(1, 4)])
        nd.memory_mb = int(MEM_CHOICES[rng.integers(1, 4)])
        if rng.random() < 0.6:
            inst = 4 if rng.random() < 0.5 else 8
            model = models[int(rng.integers(0, 3))]
            nd.devices = [DeviceGroup("nvidia", "gpu", model, inst, dict(GPU_MODELS[model]))]
            held = int(rng.integers(0, inst + 1))
            if busy > 0.0 and rng.random() < busy:
                held = inst
            j = 0
            while held > 0:
                take = min(held, int(rng.integers(1, 5)))
                allocs.append(Allocation(node_id=nid, job_id="batch-%d" % (k % 31), task_group="train",
                                         cpu_shares=500, memory_mb=1024, disk_mb=300, priority=20,
                                         devices=[(0, take)], max_parallel=(k % 3)))
                held -= take
                j += 1
        nd.compute_class()
        nodes.append(nd)
    return nodes, allocs


def job_c5(count: int = 1000) -> Job:
    """Priority-80 service job: two GPUs with >= 40 GiB each, affinity for h100."""
    return Job(
        id="svc-c5", priority=80, datacenters=["dc1"],
        constraints=[Constraint("${attr.kernel.name}", "linux", "=")],
        task_groups=[TaskGroup(name="infer", count=count, ephemeral_disk_mb=150, tasks=[
            Task(name="infer", driver="exec", cpu=1000, memory_mb=2048,
                 devices=[RequestedDevice("nvidia/gpu", 2,
                                          constraints=[Constraint("${device.attr.memory}", "40 GiB", ">=")],
                                          affinities=[Affinity("${device.model}", "h100", "=", 50)])])])],
    )
