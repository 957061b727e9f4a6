"""Host-side mirror of the reference domain types the placement path reads.

Field names follow nomad/structs/structs.go so the parity tests read like the
reference's own tests (scheduler/*_test.go). Only the fields the placement
stack consults are modelled:

  Node            structs.go:1812-1914 (+ NodeResources 2700-2852, ReservedResources)
  Allocation      structs.go:9180-9341 (ComparableResources flattened)
  Job/TaskGroup/Task, Constraint, Affinity, Spread/SpreadTarget, NetworkResource
  SchedulerConfiguration (operator.go:128-210)

`compute_class` restates Node.ComputeClass (node_class.go:31-104): a hash over
Datacenter, Attributes and Meta without `unique.` keys, NodeClass and device
identity/attributes. Only the partition it induces matters;
the hash value itself is unpinned.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple


@dataclass
class DriverInfo:
    detected: bool = True
    healthy: bool = True


@dataclass
class NetworkResource:
    """NodeResources.Networks entry (node side) or a network ask (job side)."""
    mode: str = "host"
    device: str = ""
    cidr: str = ""
    ip: str = ""
    mbits: int = 0
    dynamic_ports: int = 0          # number of DynamicPorts in an ask
    reserved_ports: List[int] = field(default_factory=list)
    port_labels: List[str] = field(default_factory=list)   # Port.Label of each reserved port (ask side)
    host_network: str = "default"   # Port.HostNetwork after Canonicalize()


@dataclass
class DeviceGroup:
    vendor: str
    type: str
    name: str
    healthy: int
    attributes: Dict[str, object] = field(default_factory=dict)


@dataclass
class Node:
    id: str
    name: str = "foobar"
    datacenter: str = "dc1"
    node_class: str = ""
    attributes: Dict[str, str] = field(default_factory=dict)
    meta: Dict[str, str] = field(default_factory=dict)
    drivers: Dict[str, DriverInfo] = field(default_factory=dict)
    cpu_shares: int = 4000
    memory_mb: int = 8192
    disk_mb: int = 100 * 1024
    reserved_cpu: int = 0
    reserved_memory_mb: int = 0
    reserved_disk_mb: int = 0
    networks: List[NetworkResource] = field(default_factory=list)
    host_network_aliases: List[str] = field(default_factory=list)
    reserved_host_ports: List[int] = field(default_factory=list)
    host_volumes: Dict[str, bool] = field(default_factory=dict)   # name -> read only
    devices: List[DeviceGroup] = field(default_factory=list)
    reservable_cores: List[int] = field(default_factory=list)   # NodeResources.Cpu.ReservableCpuCores
    total_cores: int = 0                                        # NodeResources.Cpu.TotalCpuCores
    reserved_cores: List[int] = field(default_factory=list)     # ReservedResources.Cpu.ReservedCpuCores
    # NodeNetworks[*].Addresses[*]: (alias, address, ReservedPorts spec); empty:
    # one address per host_network_aliases entry at the first network's IP
    addresses: List[Tuple[str, str, str]] = field(default_factory=list)
    status: str = "ready"
    drain: bool = False
    eligible: bool = True
    computed_class: str = ""

    def node_addresses(self) -> List[Tuple[str, str, str]]:
        """NodeNetworks addresses (alias, address, ReservedPorts spec) in node order."""
        if self.addresses:
            return list(self.addresses)
        ip = ""
        for w in self.networks:
            ip = w.ip or (w.cidr.split("/")[0] if w.cidr else "")
            if ip:
                break
        return [(a, ip, "") for a in self.host_network_aliases]

    def ready(self) -> bool:
        """Node.Ready (structs.go:1935-1937)."""
        return self.status == "ready" and not self.drain and self.eligible

    def compute_class(self) -> str:
        h = hashlib.blake2b(digest_size=8)

        def put(s):
            h.update(s.encode())
            h.update(b"\0")

        put(self.datacenter)
        for k in sorted(self.attributes):
            if not k.startswith("unique."):
                put(k); put(self.attributes[k])
        put("|meta")
        for k in sorted(self.meta):
            if not k.startswith("unique."):
                put(k); put(self.meta[k])
        put("|class"); put(self.node_class)
        for d in self.devices:
            put(d.vendor); put(d.type); put(d.name)
            for k in sorted(d.attributes):   # NodeDeviceResource.HashIncludeMap: no unique.* keys
                if not k.startswith("unique."):
                    put(k); put(repr(d.attributes[k]))
        self.computed_class = "v1:%d" % int.from_bytes(h.digest(), "little")
        return self.computed_class


def escaped_constraints(constraints):
    """EscapedConstraints (node_class.go:108-132): the constraints whose LTarget
    or RTarget escapes the computed class (${node.unique.*}, ${attr.unique.*},
    ${meta.unique.*})."""
    def escapes(t):
        return t.startswith("${node.unique.") or t.startswith("${attr.unique.") or t.startswith("${meta.unique.")
    return [c for c in constraints if escapes(c.ltarget) or escapes(c.rtarget)]


@dataclass
class Allocation:
    node_id: str
    job_id: str
    task_group: str
    namespace: str = "default"
    cpu_shares: int = 0
    memory_mb: int = 0
    disk_mb: int = 0
    net_mbits: int = 0
    has_network: Optional[bool] = None   # Flattened.Networks non-empty (None: net_mbits/dyn_ports/ports > 0)
    net_device: Optional[str] = None     # NetworkResource.Device (None: the node's first device network)
    dyn_ports: int = 0
    priority: int = 50
    terminal: bool = False
    # (device group index on the node, healthy instances held): AllocatedDeviceResource
    # DeviceIDs counted per group (nomad/structs/devices.go:62-100)
    devices: List[Tuple[int, int]] = field(default_factory=list)
    max_parallel: int = 0         # TaskGroup.Migrate.MaxParallel of the alloc's job (preemption.go:146-150)
    reserved_cores: List[int] = field(default_factory=list)   # Flattened.Cpu.ReservedCores
    ports: List[Tuple[str, int]] = field(default_factory=list)   # (HostIP, port) the alloc holds


@dataclass
class Constraint:
    ltarget: str = ""
    rtarget: str = ""
    operand: str = "="

    def __str__(self):   # Constraint.String (structs.go:8292)
        return "%s %s %s" % (self.ltarget, self.operand, self.rtarget)


@dataclass
class Affinity:
    ltarget: str = ""
    rtarget: str = ""
    operand: str = "="
    weight: int = 50


@dataclass
class SpreadTarget:
    value: str
    percent: int


@dataclass
class Spread:
    attribute: str
    weight: int = 50
    targets: List[SpreadTarget] = field(default_factory=list)


@dataclass
class RequestedDevice:
    """structs.RequestedDevice (structs.go:2700-2761): name is vendor/type/model,
    vendor/type or type."""
    name: str = "gpu"
    count: int = 1
    constraints: List[Constraint] = field(default_factory=list)
    affinities: List[Affinity] = field(default_factory=list)


@dataclass
class Task:
    name: str = "web"
    driver: str = "exec"
    cpu: int = 500
    memory_mb: int = 256
    memory_max_mb: int = 0
    cores: int = 0
    lifecycle: int = 0            # abi.PE_LC_*
    network: Optional[NetworkResource] = None
    constraints: List[Constraint] = field(default_factory=list)
    affinities: List[Affinity] = field(default_factory=list)
    devices: List[RequestedDevice] = field(default_factory=list)


@dataclass
class TaskGroup:
    name: str = "web"
    count: int = 1
    ephemeral_disk_mb: int = 150
    constraints: List[Constraint] = field(default_factory=list)
    affinities: List[Affinity] = field(default_factory=list)
    spreads: List[Spread] = field(default_factory=list)
    tasks: List[Task] = field(default_factory=list)
    network: Optional[NetworkResource] = None
    host_volumes: List[tuple] = field(default_factory=list)   # (source, read_only)


@dataclass
class Job:
    id: str
    namespace: str = "default"
    type: int = 0                 # abi.PE_JOB_*
    priority: int = 50
    version: int = 0
    datacenters: List[str] = field(default_factory=lambda: ["dc1"])
    constraints: List[Constraint] = field(default_factory=list)
    affinities: List[Affinity] = field(default_factory=list)
    spreads: List[Spread] = field(default_factory=list)
    task_groups: List[TaskGroup] = field(default_factory=list)


@dataclass
class SchedulerConfig:
    algorithm: str = "binpack"    # binpack | spread
    memory_oversubscription: bool = False
    preempt_system: bool = False
    preempt_service: bool = False
