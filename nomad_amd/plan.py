"""Plan applier fit check: host mirror of the reference's plan evaluation.

Reference (leader side): evaluatePlanPlacements and evaluateNodePlan
(nomad/plan_apply.go:439-674) → structs.AllocsFit(node, proposed, nil, true)
(nomad/structs/funcs.go:148-211). `Planner` keeps the state snapshot resident
on the GPU (pe_planner_set_state), evaluates every node of a plan in one
kernel (pe_planner_evaluate) and folds an applied plan back into the snapshot
(pe_planner_commit, the optimistic UpsertPlanResults of planApply,
plan_apply.go:207). Method names follow the reference: `evaluate_node_plan`
returns (fit, reason) like evaluateNodePlan; `evaluate_plan_placements`
returns a PlanResult like evaluatePlanPlacements.

The dataclasses model the structs.Node / structs.Allocation / structs.Plan
fields this path reads. There is no CPU fallback: the Planner raises when the
HIP library or a device is missing. oracle/plan_apply.py is the CPU
restatement used only by the tests and the bench baseline.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .encode import Interner

# ---- domain types (field names follow nomad/structs/structs.go) -------------


@dataclass
class NodeNetworkAddress:          # structs.NodeNetworkAddress
    address: str
    alias: str = "default"
    reserved_ports: str = ""       # ReservedPorts spec, ParsePortRanges syntax


@dataclass
class NodeDevice:                  # structs.NodeDevice
    id: str
    healthy: bool = True


@dataclass
class NodeDeviceResource:          # structs.NodeDeviceResource (DeviceIdTuple + instances)
    vendor: str
    type: str
    name: str
    instances: List[NodeDevice] = field(default_factory=list)


@dataclass
class PlanNode:
    """structs.Node as the plan applier reads it (NodeResources 0.9+ layout)."""
    id: str
    status: str = "ready"                     # NodeStatusReady
    scheduling_eligibility: str = "eligible"  # NodeSchedulingEligible / "ineligible"
    cpu_shares: int = 4000
    memory_mb: int = 8192
    disk_mb: int = 100 * 1024
    reserved_cpu: int = 0                     # ReservedResources (None ⇒ 0)
    reserved_memory_mb: int = 0
    reserved_disk_mb: int = 0
    reservable_cores: List[int] = field(default_factory=list)   # NodeResources.Cpu.ReservableCpuCores
    reserved_cores: List[int] = field(default_factory=list)     # ReservedResources.Cpu.ReservedCpuCores
    networks: List[Tuple[str, str]] = field(default_factory=list)   # NodeResources.Networks: (Device, IP)
    addresses: List[NodeNetworkAddress] = field(default_factory=list)  # NodeNetworks[*].Addresses
    reserved_host_ports: str = ""             # ReservedResources.Networks.ReservedHostPorts
    devices: List[NodeDeviceResource] = field(default_factory=list)


@dataclass
class Port:                        # structs.AllocatedPortMapping (Shared.Ports)
    value: int
    host_ip: str


@dataclass
class AllocNetwork:                # structs.NetworkResource of an alloc
    ip: str
    device: str = ""
    mbits: int = 0
    reserved_ports: List[int] = field(default_factory=list)
    dynamic_ports: List[int] = field(default_factory=list)


@dataclass
class AllocDevice:                 # structs.AllocatedDeviceResource
    vendor: str
    type: str
    name: str
    device_ids: List[str] = field(default_factory=list)


@dataclass
class PlanAlloc:
    """structs.Allocation as AllocsFit reads it; resources are
    ComparableResources() (structs.go:9656-9688), flattened by the caller."""
    id: str
    node_id: str
    desired_status: str = "run"
    client_status: str = "pending"
    cpu_shares: int = 500
    memory_mb: int = 256
    disk_mb: int = 150
    reserved_cores: List[int] = field(default_factory=list)
    shared_ports: List[Port] = field(default_factory=list)            # AllocatedResources.Shared.Ports
    shared_networks: List[AllocNetwork] = field(default_factory=list)  # AllocatedResources.Shared.Networks
    task_networks: Dict[str, List[AllocNetwork]] = field(default_factory=dict)  # Tasks[t].Networks
    devices: List[AllocDevice] = field(default_factory=list)          # Tasks[*].Devices

    def terminal(self) -> bool:
        """Allocation.TerminalStatus (structs.go:9341-9365)."""
        return self.desired_status in ("stop", "evict") or self.client_status in ("complete", "failed", "lost")

    def marked_ports(self) -> List[Tuple[str, int]]:
        """The (IP, port) pairs NetworkIndex.AddAllocs marks (network.go:144-193)."""
        if self.shared_ports:
            return [(p.host_ip, p.value) for p in self.shared_ports]
        out = []
        nets = list(self.shared_networks)
        for t in self.task_networks.values():
            if t:
                nets.append(t[0])
        for n in nets:
            out.extend((n.ip, v) for v in list(n.reserved_ports) + list(n.dynamic_ports))
        return out


@dataclass
class Plan:                        # structs.Plan (the maps evaluatePlanPlacements reads)
    node_update: Dict[str, List[PlanAlloc]] = field(default_factory=dict)
    node_allocation: Dict[str, List[PlanAlloc]] = field(default_factory=dict)
    node_preemptions: Dict[str, List[PlanAlloc]] = field(default_factory=dict)
    all_at_once: bool = False

    def node_ids(self) -> List[str]:
        """nodeIDList: NodeUpdate keys, then NodeAllocation keys not seen (plan_apply.go:451-464)."""
        seen, out = set(), []
        for k in list(self.node_update) + list(self.node_allocation):
            if k not in seen:
                seen.add(k)
                out.append(k)
        return out


@dataclass
class PlanResult:                  # structs.PlanResult (the parts decided here)
    node_update: Optional[Dict[str, List[PlanAlloc]]]
    node_allocation: Optional[Dict[str, List[PlanAlloc]]]
    node_preemptions: Optional[Dict[str, List[PlanAlloc]]]
    partial_commit: bool
    reasons: Dict[str, str]        # node id -> evaluateNodePlan reason ("" when it fits)


def reason_string(code: int) -> str:
    return abi.PLAN_REASONS[code]


def assemble_result(plan: Plan, node_ids: Sequence[str], fits: Sequence[bool], reasons: Sequence[str],
                    snapshot_alloc) -> PlanResult:
    """evaluatePlanPlacements' handleResult over per-node outcomes
    (plan_apply.go:471-526): AllAtOnce empties the result on the first misfit;
    preemptions are kept only if the alloc still exists and is not terminal.
    `snapshot_alloc(id)` returns the snapshot's PlanAlloc or None."""
    res = PlanResult({}, {}, {}, False, {})
    for nid, ok, why in zip(node_ids, fits, reasons):
        res.reasons[nid] = why
        if not ok:
            res.partial_commit = True
            if plan.all_at_once:
                res.node_update = res.node_allocation = res.node_preemptions = None
                return res
            continue
        if plan.node_update.get(nid):
            res.node_update[nid] = plan.node_update[nid]
        if plan.node_allocation.get(nid):
            res.node_allocation[nid] = plan.node_allocation[nid]
        if nid in plan.node_preemptions and plan.node_preemptions[nid] is not None:
            keep = []
            for a in plan.node_preemptions[nid]:
                cur = snapshot_alloc(a.id)
                if cur is not None and not cur.terminal():
                    keep.append(a)
            res.node_preemptions[nid] = keep
    return res


# ---- flattening into the pe_plan_* tables -----------------------------------


def _arr(x, dt):
    return np.ascontiguousarray(np.asarray(x, dtype=dt))


def _p(a, t):
    return a.ctypes.data_as(t)


def _csr(items_per_row, conv_list):
    """items_per_row: list of lists of tuples; returns (off, [col arrays])."""
    off = np.zeros(len(items_per_row) + 1, dtype=np.uint32)
    np.cumsum([len(x) for x in items_per_row], out=off[1:])
    cols = []
    flat = [t for row in items_per_row for t in row]
    for k, dt in enumerate(conv_list):
        cols.append(_arr([t[k] for t in flat] if flat else [], dt))
    return off, cols


def encode_nodes(nodes: Sequence[PlanNode], it: Interner):
    keep = []
    I = it.intern
    t = abi.pe_plan_node_table()
    t.n = len(nodes)

    def col(vals, dt, ptr):
        a = _arr(vals, dt)
        keep.append(a)
        return _p(a, ptr)

    t.ready = col([n.status == "ready" for n in nodes], np.uint8, abi.u8p)
    t.eligible = col([n.scheduling_eligibility != "ineligible" for n in nodes], np.uint8, abi.u8p)
    t.cpu_shares = col([n.cpu_shares for n in nodes], np.int64, abi.i64p)
    t.memory_mb = col([n.memory_mb for n in nodes], np.int64, abi.i64p)
    t.disk_mb = col([n.disk_mb for n in nodes], np.int64, abi.i64p)
    t.reserved_cpu = col([n.reserved_cpu for n in nodes], np.int64, abi.i64p)
    t.reserved_memory_mb = col([n.reserved_memory_mb for n in nodes], np.int64, abi.i64p)
    t.reserved_disk_mb = col([n.reserved_disk_mb for n in nodes], np.int64, abi.i64p)
    # available cores = ReservableCpuCores − ReservedCpuCores (cpuset Difference)
    cores = [[(c,) for c in sorted(set(n.reservable_cores) - set(n.reserved_cores))] for n in nodes]
    off, (cid,) = _csr(cores, [np.uint32])
    keep += [off, cid]
    t.core_off, t.core_id = _p(off, abi.u32p), _p(cid, abi.u32p)
    nets = [[(I(ip),) for dev, ip in n.networks if dev != ""] for n in nodes]
    off, (nip,) = _csr(nets, [np.uint32])
    keep += [off, nip]
    t.net_off, t.net_ip = _p(off, abi.u32p), _p(nip, abi.u32p)
    addrs = [[(I(a.address), I(a.reserved_ports)) for a in n.addresses] for n in nodes]
    off, (aip, arp) = _csr(addrs, [np.uint32, np.uint32])
    keep += [off, aip, arp]
    t.addr_off, t.addr_ip, t.addr_reserved_ports = _p(off, abi.u32p), _p(aip, abi.u32p), _p(arp, abi.u32p)
    t.reserved_host_ports = col([I(n.reserved_host_ports) for n in nodes], np.uint32, abi.u32p)
    groups = [[(I(d.vendor), I(d.type), I(d.name)) for d in n.devices] for n in nodes]
    off, (dv, dt_, dn) = _csr(groups, [np.uint32, np.uint32, np.uint32])
    inst = [[(I(i.id), 1 if i.healthy else 0) for i in d.instances] for n in nodes for d in n.devices]
    ioff, (iid, ih) = _csr(inst, [np.uint32, np.uint8])
    keep += [off, dv, dt_, dn, ioff, iid, ih]
    t.dev_off, t.dev_vendor, t.dev_type, t.dev_name = (_p(off, abi.u32p), _p(dv, abi.u32p), _p(dt_, abi.u32p),
                                                       _p(dn, abi.u32p))
    t.inst_off, t.inst_id, t.inst_healthy = _p(ioff, abi.u32p), _p(iid, abi.u32p), _p(ih, abi.u8p)
    return t, keep


def encode_allocs(allocs: Sequence[PlanAlloc], it: Interner, rows: Optional[Sequence[int]] = None):
    keep = []
    I = it.intern
    t = abi.pe_plan_alloc_table()
    t.count = len(allocs)

    def col(vals, dt, ptr):
        a = _arr(vals, dt)
        keep.append(a)
        return _p(a, ptr)

    t.node_row = col(rows if rows is not None else [abi.PE_NONE] * len(allocs), np.uint32, abi.u32p)
    t.terminal = col([a.terminal() for a in allocs], np.uint8, abi.u8p)
    t.cpu_shares = col([a.cpu_shares for a in allocs], np.int64, abi.i64p)
    t.memory_mb = col([a.memory_mb for a in allocs], np.int64, abi.i64p)
    t.disk_mb = col([a.disk_mb for a in allocs], np.int64, abi.i64p)
    off, (cid,) = _csr([[(c,) for c in a.reserved_cores] for a in allocs], [np.uint32])
    keep += [off, cid]
    t.core_off, t.core_id = _p(off, abi.u32p), _p(cid, abi.u32p)
    off, (pip, pv) = _csr([[(I(ip), v) for ip, v in a.marked_ports()] for a in allocs], [np.uint32, np.int64])
    keep += [off, pip, pv]
    t.port_off, t.port_ip, t.port_value = _p(off, abi.u32p), _p(pip, abi.u32p), _p(pv, abi.i64p)
    devs = [[(I(d.vendor), I(d.type), I(d.name), I(i)) for d in a.devices for i in d.device_ids] for a in allocs]
    off, (dv, dt_, dn, di) = _csr(devs, [np.uint32] * 4)
    keep += [off, dv, dt_, dn, di]
    t.dev_off, t.dev_vendor, t.dev_type, t.dev_name, t.dev_instance = (
        _p(off, abi.u32p), _p(dv, abi.u32p), _p(dt_, abi.u32p), _p(dn, abi.u32p), _p(di, abi.u32p))
    return t, keep


class EncodedPlan:
    """A Plan flattened against a snapshot (node rows, snapshot alloc indices)."""

    def __init__(self, plan: Plan, row_of: Dict[str, int], alloc_index: Dict[str, int],
                 interner: Optional[Interner] = None):
        self.plan = plan
        self.node_ids = plan.node_ids()
        it = interner if interner is not None else Interner()
        rows, rm_items, placed = [], [], []
        for nid in self.node_ids:
            rows.append(row_of.get(nid, abi.PE_NONE))
            rm = []
            for m in (plan.node_update, plan.node_preemptions, plan.node_allocation):
                for a in m.get(nid) or []:
                    j = alloc_index.get(a.id)
                    if j is not None:
                        rm.append((j,))
            rm_items.append(rm)
            placed.append(plan.node_allocation.get(nid) or [])
        self.rows = _arr(rows, np.uint32)
        rm_off, (rm_idx,) = _csr(rm_items, [np.uint32])
        self.place_off = np.zeros(len(placed) + 1, dtype=np.uint32)
        np.cumsum([len(x) for x in placed], out=self.place_off[1:])
        self.flat_allocs = [a for x in placed for a in x]
        at, akeep = encode_allocs(self.flat_allocs, it)
        st, skeep = it.table()
        self.keep = [rm_off, rm_idx, akeep, skeep]
        self.strtab = st
        self.c = abi.pe_plan(len(self.node_ids), _p(self.rows, abi.u32p), _p(rm_off, abi.u32p),
                             _p(rm_idx, abi.u32p), _p(self.place_off, abi.u32p), at)


class PlannerError(RuntimeError):
    pass


class Planner:
    """Resident-snapshot plan evaluator over the HIP library (pe_planner_*)."""

    def __init__(self, device: int = 0):
        from .stack import load_engine
        self.lib = abi.bind_planner(load_engine())
        self.h = self.lib.pe_planner_create(device)
        if not self.h:
            raise PlannerError("pe_planner_create failed: no HIP device %d" % device)
        self.nodes: List[PlanNode] = []
        self.row_of: Dict[str, int] = {}
        self.allocs: List[PlanAlloc] = []
        self.alloc_index: Dict[str, int] = {}   # live alloc id -> snapshot index
        self.interner = Interner()

    def close(self):
        if getattr(self, "h", None):
            self.lib.pe_planner_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc != 0:
            raise PlannerError("%s (code %d)" % (self.lib.pe_planner_last_error(self.h).decode(), rc))

    def set_state(self, nodes: Sequence[PlanNode], allocs: Sequence[PlanAlloc] = ()):
        """Snapshot: nodes and their allocations (state.AllocsByNode)."""
        self.nodes = list(nodes)
        self.row_of = {n.id: i for i, n in enumerate(self.nodes)}
        self.allocs = list(allocs)
        self.alloc_index = {a.id: i for i, a in enumerate(self.allocs)}
        # one growing string table for the snapshot and every later plan: the
        # library then maps only the strings a call adds
        import time
        t0 = time.perf_counter()
        self.interner = it = Interner()
        nt, nk = encode_nodes(self.nodes, it)
        at, ak = encode_allocs(self.allocs, it, [self.row_of[a.node_id] for a in self.allocs])
        st, sk = it.table()
        t1 = time.perf_counter()
        self._check(self.lib.pe_planner_set_state(self.h, C.byref(st), C.byref(nt), C.byref(at)))
        # (the Python flattening, the pe_planner_set_state call on the flat arrays) in seconds
        self.last_set_state_split = (t1 - t0, time.perf_counter() - t1)

    def snapshot_alloc(self, alloc_id: str) -> Optional[PlanAlloc]:
        j = self.alloc_index.get(alloc_id)
        return None if j is None else self.allocs[j]

    def encode(self, plan: Plan) -> EncodedPlan:
        return EncodedPlan(plan, self.row_of, self.alloc_index, self.interner)

    def evaluate(self, ep: EncodedPlan) -> np.ndarray:
        """Per-node PE_PLAN_* codes in ep.node_ids order (one kernel launch)."""
        reason = np.zeros(max(len(ep.node_ids), 1), dtype=np.uint8)
        n_fit = C.c_uint32(0)
        self._check(self.lib.pe_planner_evaluate(self.h, C.byref(ep.strtab), C.byref(ep.c),
                                                 _p(reason, abi.u8p), C.byref(n_fit)))
        return reason[:len(ep.node_ids)]

    def kernel_ms(self) -> float:
        return self.lib.pe_planner_kernel_ms(self.h)

    def last_bytes(self) -> int:
        return self.lib.pe_planner_last_bytes(self.h)

    def evaluate_node_plan(self, plan: Plan, node_id: str) -> Tuple[bool, str]:
        """evaluateNodePlan (plan_apply.go:611-674) for one node."""
        sub = Plan({node_id: plan.node_update.get(node_id) or []} if node_id in plan.node_update else {},
                   {node_id: plan.node_allocation[node_id]} if node_id in plan.node_allocation else {},
                   {node_id: plan.node_preemptions[node_id]} if node_id in plan.node_preemptions else {})
        ep = self.encode(sub)
        if not ep.node_ids:   # node in neither map: nothing placed ⇒ evict-only fit
            return True, ""
        code = int(self.evaluate(ep)[0])
        return code == abi.PE_PLAN_FIT, reason_string(code)

    def evaluate_plan_placements(self, plan: Plan, ep: Optional[EncodedPlan] = None) -> PlanResult:
        """evaluatePlanPlacements (plan_apply.go:439-582) minus the refresh-index
        and deployment bookkeeping (state-store work)."""
        ep = ep or self.encode(plan)
        codes = self.evaluate(ep)
        return assemble_result(plan, ep.node_ids, [c == abi.PE_PLAN_FIT for c in codes],
                               [reason_string(int(c)) for c in codes], self.snapshot_alloc)

    def apply(self, plan: Plan, result: PlanResult, ep: Optional[EncodedPlan] = None):
        """Fold an applied PlanResult into the resident snapshot: its NodeUpdate /
        NodePreemptions / replaced allocs stop counting, its NodeAllocation allocs
        are appended (state.UpsertPlanResults)."""
        ep = ep or self.encode(plan)
        applied = set(result.node_allocation or {}) | set(result.node_update or {}) | \
            set(result.node_preemptions or {})
        keep = _arr([nid in applied for nid in ep.node_ids] or [0], np.uint8)
        self._check(self.lib.pe_planner_commit(self.h, C.byref(ep.strtab), C.byref(ep.c), _p(keep, abi.u8p)))
        for i, nid in enumerate(ep.node_ids):
            if not keep[i]:
                continue
            for m in (plan.node_update, plan.node_preemptions, plan.node_allocation):
                for a in m.get(nid) or []:
                    self.alloc_index.pop(a.id, None)
            for a in plan.node_allocation.get(nid) or []:
                self.alloc_index[a.id] = len(self.allocs)
                self.allocs.append(a)
