"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke, bench.py's
cpu_baseline leg). The product never imports this module.

CPU restatement of the plan applier's fit check, following the reference
function by function on the nomad_amd.plan dataclasses (plain data):

  evaluatePlanPlacements      nomad/plan_apply.go:439-582 (handleResult 471-526)
  evaluateNodePlan            nomad/plan_apply.go:611-674
  RemoveAllocs                nomad/structs/funcs.go:47-64
  AllocsFit                   nomad/structs/funcs.go:148-211
  ComparableResources.Superset nomad/structs/structs.go:3891-3905
  NetworkIndex.SetNode        nomad/structs/network.go:92-141
  NetworkIndex.AddAllocs      nomad/structs/network.go:144-193
  AddReserved / AddReservedPorts / AddReservedPortRange / AddReservedPortsForIP
                              nomad/structs/network.go:196-296
  ParsePortRanges             nomad/structs/funcs.go:495-548
  DeviceAccounter             nomad/structs/devices.go:22-101
  Allocation.TerminalStatus   nomad/structs/structs.go:9341-9365

Go map iteration order is unspecified; where it could matter (ParsePortRanges
returns map keys, AddReserved* return early on an invalid port) this restatement
walks ports ascending, which is one legal order. Pinned by the reference's own
tests in nomad/plan_apply_test.go:392-987 (tests/test_plan_apply.py).
"""
from __future__ import annotations

MAX_VALID_PORT = 65536   # network.go:22


def terminal_status(a) -> bool:
    return a.desired_status in ("stop", "evict") or a.client_status in ("complete", "failed", "lost")


def _parse_uint(s):
    if not s or any(c < "0" or c > "9" for c in s):
        raise ValueError(s)
    v = int(s)
    if v >= 1 << 64:
        raise ValueError(s)
    return v


def parse_port_ranges(spec: str):
    parts = spec.split(",")
    if len(parts) == 1 and parts[0] == "":
        return []
    ports = set()
    for part in parts:
        part = part.strip(" \t\n\r\v\f")
        rp = part.split("-")
        if len(rp) == 1:
            if rp[0] == "":
                raise ValueError("can't specify empty port")
            ports.add(_parse_uint(rp[0]))
        elif len(rp) == 2:
            start, end = _parse_uint(rp[0]), _parse_uint(rp[1])
            if end < start:
                raise ValueError("invalid range")
            # ports >= 65536 only ever hit the `port >= maxValidPort` guard
            for i in range(start, min(end, MAX_VALID_PORT) + 1):
                ports.add(i)
        else:
            raise ValueError("can only parse single port numbers or port ranges")
    return sorted(ports)


class NetworkIndex:
    def __init__(self):
        self.avail_networks = []      # (device, ip)
        self.used_ports = {}          # ip -> set(ports)

    def _used(self, ip):
        return self.used_ports.setdefault(ip, set())

    def overcommitted(self):
        return False                  # network.go:79-90: bandwidth check disabled

    def set_node(self, node) -> bool:
        for dev, ip in node.networks:
            if dev != "":
                self.avail_networks.append((dev, ip))
        collide = False
        for a in node.addresses:
            if self.add_reserved_ports_for_ip(a.reserved_ports, a.address):
                collide = True
        if node.reserved_host_ports != "":
            collide = self.add_reserved_port_range(node.reserved_host_ports)
        return collide

    def add_reserved_ports_for_ip(self, spec, ip) -> bool:
        try:
            ports = parse_port_ranges(spec)
        except ValueError:
            return False
        used = self._used(ip)
        collide = False
        for p in ports:
            if p >= MAX_VALID_PORT:
                return True
            if p in used:
                collide = True
            else:
                used.add(p)
        return collide

    def add_reserved_port_range(self, spec) -> bool:
        try:
            ports = parse_port_ranges(spec)
        except ValueError:
            return False
        for _, ip in self.avail_networks:
            self._used(ip)
        collide = False
        for used in self.used_ports.values():
            for p in ports:
                if p >= MAX_VALID_PORT:
                    return True
                if p in used:
                    collide = True
                else:
                    used.add(p)
        return collide

    def _mark(self, ip, ports) -> bool:
        used = self._used(ip)
        collide = False
        for v in ports:
            if v < 0 or v >= MAX_VALID_PORT:
                return True
            if v in used:
                collide = True
            else:
                used.add(v)
        return collide

    def add_allocs(self, allocs) -> bool:
        collide = False
        for a in allocs:
            if terminal_status(a):
                continue
            if a.shared_ports:
                # AddReservedPorts: early return on an invalid port
                for p in a.shared_ports:
                    if p.value < 0 or p.value >= MAX_VALID_PORT:
                        collide = True
                        break
                    used = self._used(p.host_ip)
                    if p.value in used:
                        collide = True
                    else:
                        used.add(p.value)
            else:
                for n in a.shared_networks:
                    if self._mark(n.ip, list(n.reserved_ports) + list(n.dynamic_ports)):
                        collide = True
                for nets in a.task_networks.values():
                    if not nets:
                        continue
                    n = nets[0]
                    if self._mark(n.ip, list(n.reserved_ports) + list(n.dynamic_ports)):
                        collide = True
        return collide


class DeviceAccounter:
    def __init__(self, node):
        self.devices = {}
        for d in node.devices:
            inst = {}
            for i in d.instances:
                if i.healthy:
                    inst[i.id] = 0
            self.devices[(d.vendor, d.type, d.name)] = inst

    def add_allocs(self, allocs) -> bool:
        collision = False
        for a in allocs:
            if terminal_status(a):
                continue
            for d in a.devices:
                inst = self.devices.get((d.vendor, d.type, d.name))
                if inst is None:
                    continue
                for iid in d.device_ids:
                    if iid in inst:
                        if inst[iid] != 0:
                            collision = True
                        inst[iid] += 1
        return collision


def allocs_fit(node, allocs, check_devices=True):
    """AllocsFit → (fit, reason)."""
    cpu = mem = disk = 0
    used_cores = set()
    overlap = False
    for a in allocs:
        if terminal_status(a):
            continue
        cpu += a.cpu_shares
        mem += a.memory_mb
        disk += a.disk_mb
        for c in set(a.reserved_cores):
            if c in used_cores:
                overlap = True
            else:
                used_cores.add(c)
    if overlap:
        return False, "cores"
    avail_cpu = node.cpu_shares - node.reserved_cpu
    avail_mem = node.memory_mb - node.reserved_memory_mb
    avail_disk = node.disk_mb - node.reserved_disk_mb
    avail_cores = set(node.reservable_cores) - set(node.reserved_cores)
    if avail_cpu < cpu:
        return False, "cpu"
    if avail_cores and not used_cores <= avail_cores:
        return False, "cores"
    if avail_mem < mem:
        return False, "memory"
    if avail_disk < disk:
        return False, "disk"
    idx = NetworkIndex()
    if idx.set_node(node) or idx.add_allocs(allocs):
        return False, "reserved port collision"
    if idx.overcommitted():
        return False, "bandwidth exceeded"
    if check_devices and DeviceAccounter(node).add_allocs(allocs):
        return False, "device oversubscribed"
    return True, ""


def remove_allocs(allocs, remove):
    ids = {r.id for r in remove}
    return [a for a in allocs if a.id not in ids]


class Snapshot:
    """The state the plan is evaluated against (nodes by ID, allocs by node)."""

    def __init__(self, nodes, allocs):
        self.nodes = {n.id: n for n in nodes}
        self.by_node = {}
        self.by_id = {}
        for a in allocs:
            self.by_node.setdefault(a.node_id, []).append(a)
            self.by_id[a.id] = a

    def alloc_by_id(self, alloc_id):
        return self.by_id.get(alloc_id)

    def apply(self, plan, result):
        """UpsertPlanResults, as far as the fit check sees it."""
        for m in (result.node_update or {}, result.node_preemptions or {}):
            for nid, allocs in m.items():
                for a in allocs:
                    self._drop(a.id)
        for nid, allocs in (result.node_allocation or {}).items():
            for a in allocs:
                self._drop(a.id)
                self.by_node.setdefault(nid, []).append(a)
                self.by_id[a.id] = a

    def _drop(self, alloc_id):
        old = self.by_id.pop(alloc_id, None)
        if old is not None:
            lst = self.by_node.get(old.node_id, [])
            self.by_node[old.node_id] = [a for a in lst if a.id != alloc_id]


def evaluate_node_plan(snap: Snapshot, plan, node_id):
    if not plan.node_allocation.get(node_id):
        return True, ""
    node = snap.nodes.get(node_id)
    if node is None:
        return False, "node does not exist"
    if node.status != "ready":
        return False, "node is not ready for placements"
    if node.scheduling_eligibility == "ineligible":
        return False, "node is not eligible"
    existing = [a for a in snap.by_node.get(node_id, []) if not terminal_status(a)]
    remove = list(plan.node_update.get(node_id) or []) + list(plan.node_preemptions.get(node_id) or []) + \
        list(plan.node_allocation.get(node_id) or [])
    proposed = remove_allocs(existing, remove) + list(plan.node_allocation.get(node_id) or [])
    return allocs_fit(node, proposed, True)


def evaluate_plan_placements(snap: Snapshot, plan):
    """Returns (node_ids, fits, reasons) in nodeIDList order; the caller builds
    the PlanResult (nomad_amd.plan.assemble_result is plain bookkeeping, and the
    oracle tests re-check it)."""
    seen, ids = set(), []
    for k in list(plan.node_update) + list(plan.node_allocation):
        if k not in seen:
            seen.add(k)
            ids.append(k)
    fits, reasons = [], []
    for nid in ids:
        ok, why = evaluate_node_plan(snap, plan, nid)
        fits.append(ok)
        reasons.append(why)
    return ids, fits, reasons
