"""Vectorised synthetic clusters for 10^5 - 10^7 nodes (bench / roofline sizes).

Builds the pe_node_table / pe_alloc_table columns directly with numpy instead
of going through per-node Python objects (nomad_amd/synth.py), so a 2^24-node
cluster is generated in seconds. The distributions follow SURVEY.md §8d:

  kind="c3": 3 DCs 50/30/20 %, kernel linux 95 % / windows, os.version in
             {4.19.0, 5.4.0, 5.10.12, 6.1.0-rc1}, meta.rack r00-r99, node_class
             c0-c7, cpu in {4000, 8000, 16000}, mem in {8192, 16384, 32768}
  kind="c4": 1 DC, ~10 % windows (constraint-filtered), ~5 % pre-filled nodes

Every node also carries mock.Node()'s drivers (exec), host network (eth0,
1000 MBits, alias "default") and reserved resources (100 cpu / 256 MB / 4 GB).
ComputedClass is the combination of the hashed fields that vary.
Node IDs are unique strings up to 2^20 nodes; above that all nodes share one ID
string (IDs are not read by these workloads: no ${node.unique.*} targets).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .encode import Interner

VERSIONS = ["4.19.0", "5.4.0", "5.10.12", "6.1.0-rc1"]


class ColumnarState:
    def __init__(self, n: int, seed: int = 7, kind: str = "c3", prefill: float = 0.0):
        rng = np.random.Generator(np.random.PCG64(seed))
        it = self.interner = Interner()
        I = it.intern
        self.n = n
        self.keep = []
        u32 = lambda a: self._k(np.ascontiguousarray(a, dtype=np.uint32))
        i32 = lambda a: self._k(np.ascontiguousarray(a, dtype=np.int32))
        i64 = lambda a: self._k(np.ascontiguousarray(a, dtype=np.int64))
        u8 = lambda a: self._k(np.ascontiguousarray(a, dtype=np.uint8))

        if kind == "c3":
            u = rng.random(n)
            dc = np.where(u < 0.5, 0, np.where(u < 0.8, 1, 2)).astype(np.uint32)
            windows = rng.random(n) >= 0.95
            ver = rng.integers(0, 4, n).astype(np.uint32)
            rack = rng.integers(0, 100, n).astype(np.uint32)
            ncls = rng.integers(0, 8, n).astype(np.uint32)
            cpu = np.array([4000, 8000, 16000])[rng.integers(0, 3, n)]
            mem = np.array([8192, 16384, 32768])[rng.integers(0, 3, n)]
        else:
            dc = np.zeros(n, dtype=np.uint32)
            windows = rng.random(n) < 0.10
            ver = np.ones(n, dtype=np.uint32)
            rack = np.zeros(n, dtype=np.uint32)
            ncls = np.zeros(n, dtype=np.uint32)
            cpu = np.array([4000, 8000, 16000])[rng.integers(0, 3, n)]
            mem = np.full(n, 8192)
        self.dc_names = ["dc1", "dc2", "dc3"]
        dc_ids = np.array([I(x) for x in self.dc_names], dtype=np.uint32)
        cls_ids = np.array([I("c%d" % k) for k in range(8)], dtype=np.uint32)
        ver_ids = np.array([I(v) for v in VERSIONS], dtype=np.uint32)
        rack_ids = np.array([I("r%02d" % k) for k in range(100)], dtype=np.uint32)
        kern_ids = np.array([I("linux"), I("windows")], dtype=np.uint32)
        # ComputedClass over the hashed fields that vary: dc, kernel, os.version, rack, node_class
        combo = ((((dc * 2 + windows.astype(np.uint32)) * 4 + ver) * 100 + rack) * 8 + ncls)
        uniq, inv = np.unique(combo, return_inverse=True)
        cc_ids = np.array([I("v1:cc%d" % int(c)) for c in uniq], dtype=np.uint32)

        self.node_id = (lambda k: "node-%08d" % k) if n <= (1 << 20) else (lambda k: "node-shared-id")
        nt = abi.pe_node_table()
        nt.n = n
        if n <= (1 << 20):
            ids = u32([I("node-%08d" % k) for k in range(n)])
        else:
            ids = u32(np.full(n, I("node-shared-id"), dtype=np.uint32))
        nt.id = ids.ctypes.data_as(abi.u32p)
        nt.name = u32(np.full(n, I("foobar"))).ctypes.data_as(abi.u32p)
        nt.datacenter = u32(dc_ids[dc]).ctypes.data_as(abi.u32p)
        nt.node_class = u32(cls_ids[ncls]).ctypes.data_as(abi.u32p)
        nt.computed_class = u32(cc_ids[inv]).ctypes.data_as(abi.u32p)
        nt.cpu_shares = i64(cpu).ctypes.data_as(abi.i64p)
        nt.memory_mb = i64(mem).ctypes.data_as(abi.i64p)
        nt.disk_mb = i64(np.full(n, 100 * 1024)).ctypes.data_as(abi.i64p)
        nt.reserved_cpu = i64(np.full(n, 100)).ctypes.data_as(abi.i64p)
        nt.reserved_memory_mb = i64(np.full(n, 256)).ctypes.data_as(abi.i64p)
        nt.reserved_disk_mb = i64(np.full(n, 4 * 1024)).ctypes.data_as(abi.i64p)
        # attributes: kernel.name, os.version, driver.exec, arch, nomad.version
        keys = np.array([I("kernel.name"), I("os.version"), I("driver.exec"), I("arch"), I("nomad.version")],
                        dtype=np.uint32)
        K = len(keys)
        vals = np.empty((n, K), dtype=np.uint32)
        vals[:, 0] = kern_ids[windows.astype(np.int64)]
        vals[:, 1] = ver_ids[ver]
        vals[:, 2] = I("1")
        vals[:, 3] = I("x86")
        vals[:, 4] = I("0.5.0")
        nt.attr_off = u32(np.arange(n + 1, dtype=np.uint64) * K).ctypes.data_as(abi.u32p)
        nt.attr_key = u32(np.tile(keys, n)).ctypes.data_as(abi.u32p)
        nt.attr_val = u32(vals.reshape(-1)).ctypes.data_as(abi.u32p)
        nt.meta_off = u32(np.arange(n + 1)).ctypes.data_as(abi.u32p)
        nt.meta_key = u32(np.full(n, I("rack"))).ctypes.data_as(abi.u32p)
        nt.meta_val = u32(rack_ids[rack]).ctypes.data_as(abi.u32p)
        one = u32(np.arange(n + 1))
        nt.drv_off = one.ctypes.data_as(abi.u32p)
        nt.drv_name = u32(np.full(n, I("exec"))).ctypes.data_as(abi.u32p)
        nt.drv_flags = u8(np.full(n, 3)).ctypes.data_as(abi.u8p)
        nt.net_off = one.ctypes.data_as(abi.u32p)
        nt.net_mode = u32(np.full(n, I("host"))).ctypes.data_as(abi.u32p)
        nt.net_device = u32(np.full(n, I("eth0"))).ctypes.data_as(abi.u32p)
        nt.net_mbits = i32(np.full(n, 1000)).ctypes.data_as(abi.i32p)
        nt.alias_off = one.ctypes.data_as(abi.u32p)
        nt.alias_name = u32(np.full(n, I("default"))).ctypes.data_as(abi.u32p)
        nt.reserved_dyn_ports = i32(np.zeros(n)).ctypes.data_as(abi.i32p)
        zero_off = u32(np.zeros(n + 1))
        nt.hv_off = zero_off.ctypes.data_as(abi.u32p)
        empty32 = u32(np.zeros(1))
        nt.hv_name = empty32.ctypes.data_as(abi.u32p)
        nt.hv_read_only = u8(np.zeros(1)).ctypes.data_as(abi.u8p)
        nt.dev_off = zero_off.ctypes.data_as(abi.u32p)
        for f in ("dev_vendor", "dev_type", "dev_name", "dev_healthy", "dev_attr_key"):
            setattr(nt, f, empty32.ctypes.data_as(abi.u32p))
        nt.dev_attr_off = u32(np.zeros(1)).ctypes.data_as(abi.u32p)
        attrs = (abi.pe_attr * 1)()
        self.keep.append(attrs)
        nt.dev_attr_val = C.cast(attrs, C.POINTER(abi.pe_attr))
        self.node_table = nt

        # pre-filled nodes: one foreign alloc leaving 100 cpu free (exhausts a 500-cpu ask)
        filled = np.nonzero(rng.random(n) < prefill)[0].astype(np.uint32)
        m = len(filled)
        at = abi.pe_alloc_table()
        at.count = m
        at.node_row = u32(filled if m else np.zeros(1)).ctypes.data_as(abi.u32p)
        at.ns = u32(np.full(max(m, 1), I("default"))).ctypes.data_as(abi.u32p)
        at.job_id = u32(np.full(max(m, 1), I("filler"))).ctypes.data_as(abi.u32p)
        at.task_group = u32(np.full(max(m, 1), I("tg"))).ctypes.data_as(abi.u32p)
        at.terminal = u8(np.zeros(max(m, 1))).ctypes.data_as(abi.u8p)
        at.priority = i32(np.full(max(m, 1), 50)).ctypes.data_as(abi.i32p)
        at.cpu_shares = i64((cpu[filled] - 200) if m else np.zeros(1)).ctypes.data_as(abi.i64p)
        at.memory_mb = i64(np.full(max(m, 1), 1024)).ctypes.data_as(abi.i64p)
        at.disk_mb = i64(np.full(max(m, 1), 300)).ctypes.data_as(abi.i64p)
        at.net_mbits = i32(np.zeros(max(m, 1))).ctypes.data_as(abi.i32p)
        at.dyn_ports = i32(np.zeros(max(m, 1))).ctypes.data_as(abi.i32p)
        at.dev_off = u32(np.zeros(max(m, 1) + 1)).ctypes.data_as(abi.u32p)
        at.dev_group = empty32.ctypes.data_as(abi.u32p)
        at.dev_count = empty32.ctypes.data_as(abi.u32p)
        self.alloc_table = at
        self.row_of = {}

    def _k(self, a):
        self.keep.append(a)
        return a

    def strtab(self):
        t, k = self.interner.table()
        self.keep.append(k)
        return t
