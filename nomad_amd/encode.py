"""Flatten host-side structs into the POD tables of include/nomad_pe.h.

This is what the cgo shim would do on the Go side: intern
strings, lay nodes out as SoA columns with CSR maps, and describe the job as
flat arrays. The arrays are owned by the returned holder objects; the engine
and the oracle copy what they need during the call.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Sequence

import numpy as np

from . import abi
from .structs import Allocation, Job, Node

MIN_DYN, MAX_DYN = 20000, 32000


class Interner:
    """One string table per state snapshot; job strings are appended later."""

    def __init__(self):
        self.ids: Dict[str, int] = {}
        self.strs: List[str] = []
        self.intern("")

    def intern(self, s: str) -> int:
        i = self.ids.get(s)
        if i is None:
            i = len(self.strs)
            self.ids[s] = i
            self.strs.append(s)
        return i

    def table(self):
        """Build a pe_strtab over the current strings; returns (struct, keepalive)."""
        blobs = [s.encode() for s in self.strs]
        offs = np.zeros(len(blobs) + 1, dtype=np.uint32)
        np.cumsum([len(b) for b in blobs], out=offs[1:])
        data = b"".join(blobs) + b"\0"
        buf = C.create_string_buffer(data, len(data))
        t = abi.pe_strtab(C.cast(buf, C.c_char_p), offs.ctypes.data_as(abi.u32p), len(blobs))
        return t, (buf, offs)


def _ptr(a: np.ndarray, t):
    return a.ctypes.data_as(t)


def _u32(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.uint32))


def _i32(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.int32))


def _i64(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.int64))


def _u8(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.uint8))


def _u16(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.uint16))


class EncodedState:
    """pe_node_table + pe_alloc_table over one Interner."""

    def __init__(self, nodes: Sequence[Node], allocs: Sequence[Allocation], interner: Interner = None):
        self.interner = interner or Interner()
        self.nodes = list(nodes)
        self.row_of = {nd.id: i for i, nd in enumerate(nodes)}
        self.keep = []
        self.node_table = self.encode_node_table(self.nodes)
        self.alloc_table = self.encode_alloc_table(allocs)

    def update_nodes(self, nodes: Sequence[Node], index=None):
        """pe_node_table of node upserts (pe_update_nodes): nodes[i] replaces
        row index[i], or is appended when index[i] is None; the mirror's node
        list and row map follow."""
        idx = []
        for i, nd in enumerate(nodes):
            r = None if index is None else index[i]
            if r is None or r < 0:
                r = len(self.nodes)
                self.nodes.append(nd)
                idx.append(abi.PE_NONE)
            else:
                old = self.nodes[r]
                if self.row_of.get(old.id) == r and old.id != nd.id:
                    del self.row_of[old.id]
                self.nodes[r] = nd
                idx.append(r)
            self.row_of[nd.id] = r
        return self.encode_node_table(list(nodes)), _u32(idx or [0])

    def encode_node_table(self, nodes: Sequence[Node]) -> abi.pe_node_table:
        """pe_node_table of `nodes` over this state's interner (the arrays stay
        alive with this object)."""
        it = self.interner
        n = len(nodes)
        keep = self.keep

        def col(f, conv):
            a = conv([f(nd) for nd in nodes])
            keep.append(a)
            return a

        def csr(get_items, convs):
            off = np.zeros(n + 1, dtype=np.uint32)
            cols = [[] for _ in convs]
            for i, nd in enumerate(nodes):
                items = get_items(nd)
                off[i + 1] = off[i] + len(items)
                for it_ in items:
                    for c, v in zip(cols, it_):
                        c.append(v)
            arrs = [conv(c) for conv, c in zip(convs, cols)]
            keep.append(off)
            keep.extend(arrs)
            return [off] + arrs

        I = it.intern
        nt = abi.pe_node_table()
        nt.n = n
        nt.id = _ptr(col(lambda x: I(x.id), _u32), abi.u32p)
        nt.name = _ptr(col(lambda x: I(x.name), _u32), abi.u32p)
        nt.datacenter = _ptr(col(lambda x: I(x.datacenter), _u32), abi.u32p)
        nt.node_class = _ptr(col(lambda x: I(x.node_class), _u32), abi.u32p)
        nt.computed_class = _ptr(col(lambda x: I(x.computed_class or x.compute_class()), _u32), abi.u32p)
        nt.cpu_shares = _ptr(col(lambda x: x.cpu_shares, _i64), abi.i64p)
        nt.memory_mb = _ptr(col(lambda x: x.memory_mb, _i64), abi.i64p)
        nt.disk_mb = _ptr(col(lambda x: x.disk_mb, _i64), abi.i64p)
        nt.reserved_cpu = _ptr(col(lambda x: x.reserved_cpu, _i64), abi.i64p)
        nt.reserved_memory_mb = _ptr(col(lambda x: x.reserved_memory_mb, _i64), abi.i64p)
        nt.reserved_disk_mb = _ptr(col(lambda x: x.reserved_disk_mb, _i64), abi.i64p)
        off, k, v = csr(lambda x: [(I(a), I(b)) for a, b in x.attributes.items()], [_u32, _u32])
        nt.attr_off, nt.attr_key, nt.attr_val = (_ptr(a, abi.u32p) for a in (off, k, v))
        off, k, v = csr(lambda x: [(I(a), I(b)) for a, b in x.meta.items()], [_u32, _u32])
        nt.meta_off, nt.meta_key, nt.meta_val = (_ptr(a, abi.u32p) for a in (off, k, v))
        off, k, f = csr(lambda x: [(I(a), (1 if d.detected else 0) | (2 if d.healthy else 0))
                                   for a, d in x.drivers.items()], [_u32, _u8])
        nt.drv_off, nt.drv_name = _ptr(off, abi.u32p), _ptr(k, abi.u32p)
        nt.drv_flags = _ptr(f, abi.u8p)
        off, m, d, mb = csr(lambda x: [(I(w.mode if w.mode != "host" else "host"), I(w.device), w.mbits)
                                       for w in x.networks], [_u32, _u32, _i32])
        nt.net_off, nt.net_mode, nt.net_device = (_ptr(a, abi.u32p) for a in (off, m, d))
        nt.net_mbits = _ptr(mb, abi.i32p)
        # the network's IP field and the one address yieldIP gives from its
        # CIDR (AssignNetwork, network.go:294-315), PE_NONE: none / several
        off, nip, cip = csr(lambda x: [(I(w.ip) if w.ip else abi.PE_NONE, _cidr_single(w.cidr, I))
                                       for w in x.networks], [_u32, _u32])
        nt.net_ip, nt.net_cidr_ip = _ptr(nip, abi.u32p), _ptr(cip, abi.u32p)
        off, al = csr(lambda x: [(I(a),) for a in x.host_network_aliases], [_u32])
        nt.alias_off, nt.alias_name = _ptr(off, abi.u32p), _ptr(al, abi.u32p)
        nt.reserved_dyn_ports = _ptr(col(lambda x: sum(1 for p in x.reserved_host_ports
                                                       if MIN_DYN <= p <= MAX_DYN), _i32), abi.i32p)
        off, hn, hr = csr(lambda x: [(I(a), int(ro)) for a, ro in x.host_volumes.items()], [_u32, _u8])
        nt.hv_off, nt.hv_name, nt.hv_read_only = _ptr(off, abi.u32p), _ptr(hn, abi.u32p), _ptr(hr, abi.u8p)
        off, dv, dt, dn, dh = csr(lambda x: [(I(g.vendor), I(g.type), I(g.name), g.healthy)
                                             for g in x.devices], [_u32, _u32, _u32, _u32])
        nt.dev_off, nt.dev_vendor, nt.dev_type, nt.dev_name, nt.dev_healthy = (
            _ptr(a, abi.u32p) for a in (off, dv, dt, dn, dh))
        # device attributes: CSR over device groups (flattened across nodes)
        groups = [g for nd in nodes for g in nd.devices]
        aoff = np.zeros(len(groups) + 1, dtype=np.uint32)
        akeys, avals = [], []
        for gi, g in enumerate(groups):
            aoff[gi + 1] = aoff[gi] + len(g.attributes)
            for key, val in g.attributes.items():
                akeys.append(I(key))
                avals.append(encode_attr(val, it))
        akeys_a = _u32(akeys)
        avals_a = (abi.pe_attr * max(1, len(avals)))(*avals)
        keep.extend([aoff, akeys_a, avals_a])
        nt.dev_attr_off, nt.dev_attr_key = _ptr(aoff, abi.u32p), _ptr(akeys_a, abi.u32p)
        nt.dev_attr_val = C.cast(avals_a, C.POINTER(abi.pe_attr))
        # NodeNetworks addresses and the node's reserved host ports (static port asks)
        NONE = abi.PE_NONE
        off, al, ip, rp = csr(lambda x: [(I(a), I(b), I(c) if c else NONE) for a, b, c in x.node_addresses()],
                              [_u32, _u32, _u32])
        nt.addr_off, nt.addr_alias, nt.addr_ip, nt.addr_rsv_ports = (_ptr(a, abi.u32p) for a in (off, al, ip, rp))
        nt.rsv_host_ports = _ptr(col(lambda x: I(",".join(str(p) for p in x.reserved_host_ports))
                                     if x.reserved_host_ports else NONE, _u32), abi.u32p)
        if any(nd.reservable_cores or nd.reserved_cores or nd.total_cores for nd in nodes):
            off, cid = csr(lambda x: [(c,) for c in x.reservable_cores], [_u16])
            nt.core_off, nt.core_id = _ptr(off, abi.u32p), _ptr(cid, abi.u16p)
            nt.total_cores = _ptr(col(lambda x: x.total_cores, _u32), abi.u32p)
            off, rid = csr(lambda x: [(c,) for c in x.reserved_cores], [_u16])
            nt.rsv_core_off, nt.rsv_core_id = _ptr(off, abi.u32p), _ptr(rid, abi.u16p)
        return nt

    def encode_alloc_table(self, allocs: Sequence[Allocation]) -> abi.pe_alloc_table:
        """pe_alloc_table over this state's interner and node rows (the arrays
        stay alive with this object)."""
        I = self.interner.intern
        keep = self.keep
        at = abi.pe_alloc_table()
        live = [a for a in allocs]
        at.count = len(live)

        def acol(f, conv):
            a = conv([f(x) for x in live] if live else [])
            keep.append(a)
            return a
        at.node_row = _ptr(acol(lambda a: self.row_of[a.node_id], _u32), abi.u32p)
        at.ns = _ptr(acol(lambda a: I(a.namespace), _u32), abi.u32p)
        at.job_id = _ptr(acol(lambda a: I(a.job_id), _u32), abi.u32p)
        at.task_group = _ptr(acol(lambda a: I(a.task_group), _u32), abi.u32p)
        at.terminal = _ptr(acol(lambda a: int(a.terminal), _u8), abi.u8p)
        at.priority = _ptr(acol(lambda a: a.priority, _i32), abi.i32p)
        at.cpu_shares = _ptr(acol(lambda a: a.cpu_shares, _i64), abi.i64p)
        at.memory_mb = _ptr(acol(lambda a: a.memory_mb, _i64), abi.i64p)
        at.disk_mb = _ptr(acol(lambda a: a.disk_mb, _i64), abi.i64p)
        at.net_mbits = _ptr(acol(lambda a: a.net_mbits, _i32), abi.i32p)
        at.dyn_ports = _ptr(acol(lambda a: a.dyn_ports, _i32), abi.i32p)
        doff = np.zeros(len(live) + 1, dtype=np.uint32)
        dgrp, dcnt = [], []
        for i, a in enumerate(live):
            for g, c in a.devices:
                dgrp.append(g)
                dcnt.append(c)
            doff[i + 1] = len(dgrp)
        dgrp_a, dcnt_a = _u32(dgrp if dgrp else [0]), _u32(dcnt if dcnt else [0])
        keep.extend([doff, dgrp_a, dcnt_a])
        at.dev_off = _ptr(doff, abi.u32p)
        at.dev_group = _ptr(dgrp_a, abi.u32p)
        at.dev_count = _ptr(dcnt_a, abi.u32p)
        at.max_parallel = _ptr(acol(lambda a: a.max_parallel, _i32), abi.i32p)
        at.has_network = _ptr(acol(lambda a: int(bool(a.net_mbits > 0 or a.dyn_ports > 0 or a.ports)
                                                  if a.has_network is None else a.has_network), _u8), abi.u8p)
        at.net_device = _ptr(acol(lambda a: abi.PE_NONE if a.net_device is None else I(a.net_device), _u32),
                             abi.u32p)
        if any(a.ports for a in live):
            poff = np.zeros(len(live) + 1, dtype=np.uint32)
            pip, pval = [], []
            for i, a in enumerate(live):
                for h, v in a.ports:
                    pip.append(I(h))
                    pval.append(v)
                poff[i + 1] = len(pip)
            pip_a, pval_a = _u32(pip), _i32(pval)
            keep.extend([poff, pip_a, pval_a])
            at.port_off, at.port_ip, at.port_value = _ptr(poff, abi.u32p), _ptr(pip_a, abi.u32p), _ptr(pval_a, abi.i32p)
        if any(a.reserved_cores for a in live):
            coff = np.zeros(len(live) + 1, dtype=np.uint32)
            cid = []
            for i, a in enumerate(live):
                cid.extend(a.reserved_cores)
                coff[i + 1] = len(cid)
            cid_a = _u16(cid if cid else [0])
            keep.extend([coff, cid_a])
            at.core_off, at.core_id = _ptr(coff, abi.u32p), _ptr(cid_a, abi.u16p)
        return at

    def strtab(self):
        t, k = self.interner.table()
        self.keep.append(k)
        return t


def _cidr_single(cidr: str, intern) -> int:
    """The only address of a CIDR block, interned (PE_NONE when the CIDR does
    not parse or holds more than one address)."""
    import ipaddress
    try:
        net = ipaddress.ip_network(cidr, strict=False)
    except ValueError:
        return abi.PE_NONE
    if net.num_addresses != 1:
        return abi.PE_NONE
    return intern(str(net.network_address))


def encode_attr(val, it: Interner) -> abi.pe_attr:
    """psstructs.Attribute: (kind, value, unit). Accepts python scalars or (value, unit)."""
    a = abi.pe_attr()
    unit = ""
    if isinstance(val, tuple):
        val, unit = val
    a.unit = it.intern(unit)
    if isinstance(val, bool):
        a.kind, a.i = abi.PE_ATTR_BOOL, int(val)
    elif isinstance(val, int):
        a.kind, a.i = abi.PE_ATTR_INT, val
    elif isinstance(val, float):
        a.kind, a.f = abi.PE_ATTR_FLOAT, val
    else:
        a.kind, a.s = abi.PE_ATTR_STRING, it.intern(str(val))
    return a


class EncodedJob:
    """pe_job over an Interner shared with the state (strings appended)."""

    def __init__(self, job: Job, interner: Interner):
        I = interner.intern
        cons, affs, spreads, targets, tasks, tgs = [], [], [], [], [], []
        devs, dcons, daffs = [], [], []
        vol_src, vol_ro = [], []
        rport_val, rport_lab = [], []

        def add_cons(cs):
            off = len(cons)
            for c in cs:
                cons.append(abi.pe_constraint(I(c.ltarget), I(c.rtarget), I(c.operand)))
            return off, len(cs)

        def add_affs(xs):
            off = len(affs)
            for a in xs:
                affs.append(abi.pe_affinity(I(a.ltarget), I(a.rtarget), I(a.operand), a.weight))
            return off, len(xs)

        def add_spreads(xs):
            off = len(spreads)
            for sp in xs:
                toff = len(targets)
                for t in sp.targets:
                    targets.append(abi.pe_spread_target(I(t.value), t.percent))
                spreads.append(abi.pe_spread(I(sp.attribute), sp.weight, toff, len(sp.targets)))
            return off, len(xs)

        pj = abi.pe_job()
        pj.id, pj.ns, pj.type, pj.priority, pj.version = I(job.id), I(job.namespace), job.type, job.priority, job.version
        pj.constraint_off, pj.constraint_count = add_cons(job.constraints)
        pj.affinity_off, pj.affinity_count = add_affs(job.affinities)
        pj.spread_off, pj.spread_count = add_spreads(job.spreads)
        for tg in job.task_groups:
            g = abi.pe_task_group()
            g.name, g.count, g.ephemeral_disk_mb = I(tg.name), tg.count, tg.ephemeral_disk_mb
            g.constraint_off, g.constraint_count = add_cons(tg.constraints)
            g.affinity_off, g.affinity_count = add_affs(tg.affinities)
            g.spread_off, g.spread_count = add_spreads(tg.spreads)
            g.task_off = len(tasks)
            for t in tg.tasks:
                pt = abi.pe_task()
                pt.name, pt.driver = I(t.name), I(t.driver)
                pt.cpu, pt.memory_mb, pt.memory_max_mb = t.cpu, t.memory_mb, t.memory_max_mb
                pt.cores, pt.lifecycle = t.cores, t.lifecycle
                if t.network is not None:
                    pt.has_network, pt.net_mbits = 1, t.network.mbits
                    pt.net_dyn_ports, pt.net_reserved_ports = t.network.dynamic_ports, len(t.network.reserved_ports)
                    pt.rport_off = len(rport_val)
                    for k, v in enumerate(t.network.reserved_ports):
                        rport_val.append(v)
                        lab = t.network.port_labels[k] if k < len(t.network.port_labels) else ""
                        rport_lab.append(I(lab))
                pt.constraint_off, pt.constraint_count = add_cons(t.constraints)
                pt.affinity_off, pt.affinity_count = add_affs(t.affinities)
                pt.device_off, pt.device_count = len(devs), len(t.devices)
                for d in t.devices:
                    r = abi.pe_device_request()
                    r.name, r.count = I(d.name), d.count
                    r.constraint_off, r.constraint_count = len(dcons), len(d.constraints)
                    for c in d.constraints:
                        dcons.append(abi.pe_constraint(I(c.ltarget), I(c.rtarget), I(c.operand)))
                    r.affinity_off, r.affinity_count = len(daffs), len(d.affinities)
                    for a in d.affinities:
                        daffs.append(abi.pe_affinity(I(a.ltarget), I(a.rtarget), I(a.operand), a.weight))
                    devs.append(r)
                tasks.append(pt)
            g.task_count = len(tg.tasks)
            if tg.network is not None:
                g.has_network, g.net_mode = 1, I(tg.network.mode)
                g.net_dyn_ports, g.net_reserved_ports = tg.network.dynamic_ports, len(tg.network.reserved_ports)
                g.net_host_network = I(tg.network.host_network)
                g.rport_off, g.rport_count = len(rport_val), len(tg.network.reserved_ports)
                for k, v in enumerate(tg.network.reserved_ports):
                    rport_val.append(v)
                    lab = tg.network.port_labels[k] if k < len(tg.network.port_labels) else ""
                    rport_lab.append(I(lab))
            else:
                g.net_mode = I("host")
                g.net_host_network = I("default")
            g.volume_off = len(vol_src)
            for src, ro in tg.host_volumes:
                vol_src.append(I(src))
                vol_ro.append(int(ro))
            g.volume_count = len(tg.host_volumes)
            tgs.append(g)
        pj.tg_count = len(tgs)

        def arr(T, xs):
            return (T * max(1, len(xs)))(*xs)
        self._arrays = [arr(abi.pe_task_group, tgs), arr(abi.pe_task, tasks), arr(abi.pe_constraint, cons),
                        arr(abi.pe_affinity, affs), arr(abi.pe_spread, spreads),
                        arr(abi.pe_spread_target, targets), arr(abi.pe_device_request, devs),
                        arr(abi.pe_constraint, dcons), arr(abi.pe_affinity, daffs)]
        (pj.task_groups, pj.tasks, pj.constraints, pj.affinities, pj.spreads, pj.spread_targets,
         pj.devices, pj.device_constraints, pj.device_affinities) = (
            C.cast(a, C.POINTER(type(a._type_()))) for a in self._arrays)
        self._vs = _u32(vol_src if vol_src else [0])
        self._vr = _u8(vol_ro if vol_ro else [0])
        pj.volume_source = _ptr(self._vs, abi.u32p)
        pj.volume_read_only = _ptr(self._vr, abi.u8p)
        self._rv = _i32(rport_val if rport_val else [0])
        self._rl = _u32(rport_lab if rport_lab else [0])
        pj.rport_value = _ptr(self._rv, abi.i32p)
        pj.rport_label = _ptr(self._rl, abi.u32p)
        self.job = pj
        self.interner = interner

    def strtab(self):
        t, k = self.interner.table()
        self._strtab_keep = k
        return t
