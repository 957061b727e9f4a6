"""Host-side mirror of the reference `scheduler.Stack` interface over a C ABI.

`GenericStack` / `SystemStack` keep the reference's method names and argument
meaning (scheduler/stack.go:23-39): SetNodes, SetJob, Select. `Place` is the
fused count loop of GenericScheduler.computePlacements (generic_sched.go:493-649)
and `SystemPlace` the SystemScheduler one (scheduler_system.go:283-425).

The product backend is nomad_amd/libnomadpe.so (HIP, gfx950). There is no CPU
fallback: constructing an engine stack without the library or without a GPU
raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import abi
from .encode import EncodedJob, EncodedState, Interner
from .structs import Allocation, Job, Node, SchedulerConfig

_HERE = os.path.dirname(os.path.abspath(__file__))
# PE_ENGINE_LIB: an A/B build of the same sources (measurement runs only)
ENGINE_LIB = os.environ.get("PE_ENGINE_LIB") or os.path.join(_HERE, "libnomadpe.so")


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (code %d)" % (msg, code))
        self.code = code


class Unsupported(EngineError):
    pass


_engine = None


def load_engine():
    """Load the HIP engine library (fails loudly when it is missing)."""
    global _engine
    if _engine is None:
        if not os.path.exists(ENGINE_LIB):
            raise EngineError(-1, "nomad_amd/libnomadpe.so is not built: run __graft_entry__.build()")
        lib = C.CDLL(ENGINE_LIB)
        abi.bind(lib, "pe_", "pe_stack_create", "pe_stack_destroy", "pe_last_error")
        lib.pe_abi_version.restype = C.c_uint32
        lib.pe_last_kernel_ms.restype = C.c_double
        lib.pe_last_kernel_ms.argtypes = [C.c_void_p]
        lib.pe_last_sweep_bytes.restype = C.c_uint32
        lib.pe_last_sweep_bytes.argtypes = [C.c_void_p]
        lib.pe_set_kernel_split.restype = C.c_int
        lib.pe_set_kernel_split.argtypes = [C.c_void_p, C.c_int]
        lib.pe_last_kernel_split.restype = C.c_int
        lib.pe_last_kernel_split.argtypes = [C.c_void_p, abi.f64p]
        lib.pe_stage_orders.restype = C.c_int
        lib.pe_stage_orders.argtypes = [C.c_void_p, abi.u32p, C.c_uint32, C.c_uint32]
        lib.pe_place_batch.restype = C.c_int
        lib.pe_place_batch.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(abi.pe_placement), abi.u32p]
        lib.pe_batch_results.restype = C.c_int
        lib.pe_batch_results.argtypes = [C.c_void_p, C.POINTER(C.POINTER(abi.pe_placement)),
                                         C.POINTER(abi.u32p), abi.u32p, abi.u32p]
        lib.pe_last_phase_ms.restype = None
        lib.pe_last_phase_ms.argtypes = [C.c_void_p, abi.f64p]
        lib.pe_select_shard.restype = C.c_int
        lib.pe_select_shard.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                        C.POINTER(abi.pe_shard_rec)]
        lib.pe_speculation_stats.restype = C.c_int
        lib.pe_speculation_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        lib.pe_comm_unique_id.restype = C.c_int
        lib.pe_comm_unique_id.argtypes = [abi.u8p, C.c_size_t]
        lib.pe_comm_init.restype = C.c_int
        lib.pe_comm_init.argtypes = [C.c_void_p, C.c_int, C.c_int, abi.u8p]
        lib.pe_place_sharded.restype = C.c_int
        lib.pe_place_sharded.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.POINTER(abi.pe_ranked_node), abi.u32p]
        lib.pe_comm_init_host.restype = C.c_int
        lib.pe_comm_init_host.argtypes = [C.c_void_p, C.c_int, C.c_int, abi.pe_exchange_fn, C.c_void_p]
        lib.pe_last_exchange_us.restype = C.c_double
        lib.pe_last_exchange_us.argtypes = [C.c_void_p]
        lib.pe_select_merge.restype = C.c_int
        lib.pe_select_merge.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(abi.pe_shard_rec), C.c_uint32,
                                        C.POINTER(abi.pe_ranked_node)]
        _engine = lib
    return _engine


def parse_metrics(text: str) -> Dict:
    """pe_last_metrics' text (also a served record's maps in pe_spec_view) as
    {"ClassFiltered": {...}, "ConstraintFiltered": {...}, "ClassExhausted":
    {...}, "DimensionExhausted": {...}, "ScoreMetaData": [(node id, NormScore,
    {scorer: score}), ...]}."""
    names = {"CF": "ClassFiltered", "KF": "ConstraintFiltered", "CE": "ClassExhausted",
             "DE": "DimensionExhausted"}
    out = {v: {} for v in names.values()}
    out["ScoreMetaData"] = []
    for line in text.split("\n"):
        if not line:
            continue
        if line.startswith("SM\t"):   # PopulateScoreMetaData: top 5 by NormScore, descending
            _, _, node_id, norm, parts = line.split("\t")
            scores = dict((k, float(v)) for k, v in (p.split("=") for p in parts.split(",") if p))
            out["ScoreMetaData"].append((node_id, float(norm), scores))
            continue
        kind, key, cnt = line.split("\t")
        out[names[kind]][key] = int(cnt)
    return out


_KIND_NAMES = {abi.PE_METRIC_CLASS_FILTERED: "ClassFiltered", abi.PE_METRIC_CONSTRAINT_FILTERED: "ConstraintFiltered",
               abi.PE_METRIC_CLASS_EXHAUSTED: "ClassExhausted",
               abi.PE_METRIC_DIMENSION_EXHAUSTED: "DimensionExhausted"}


def decode_metrics(stack, counts, c0: int, c1: int, scores, s0: int, s1: int) -> Dict:
    """Binary AllocMetric maps (pe_metric_count[c0:c1], pe_metric_score[s0:s1])
    in parse_metrics' shape; keys resolved through pe_metric_string."""
    out = {v: {} for v in _KIND_NAMES.values()}
    out["ScoreMetaData"] = []
    cache = getattr(stack, "_mkey_cache", None)
    if cache is None:
        cache = stack._mkey_cache = {}
    for i in range(c0, c1):
        e = counts[i]
        k = cache.get(e.key)
        if k is None:
            k = cache[e.key] = stack.MetricString(e.key)
        out[_KIND_NAMES[e.kind]][k] = int(e.count)
    for i in range(s0, s1):
        m = scores[i]
        parts = {abi.SCORER_NAMES[m.scorer[j]]: float(m.score[j]) for j in range(m.n_scores)}
        nid = stack.nodes[m.row].id if stack.nodes is not None else stack.state.node_id(m.row)
        out["ScoreMetaData"].append((nid, float(m.norm), parts))
    return out


def view_metrics(stack, view, k: int) -> Dict:
    """Record k's maps from the served-Select view (pe_spec_view.mcounts / mscores)."""
    return decode_metrics(stack, view.mcounts, view.mcounts_off[k], view.mcounts_off[k + 1],
                          view.mscores, view.mscores_off[k], view.mscores_off[k + 1])


@dataclass
class SelectOptions:
    """SelectOptions (stack.go:34-39); nodes are given as node IDs or rows."""
    penalty_node_ids: Sequence[str] = ()
    preferred_nodes: Sequence[str] = ()
    preempt: bool = False
    alloc_name: str = ""


def _core_ids(mask) -> List[int]:
    """Core ids of a 256-bit pe_ranked_node.reserved_cores mask, ascending."""
    out = []
    for w in range(4):
        m = int(mask[w])
        while m:
            low = m & -m
            out.append(64 * w + low.bit_length() - 1)
            m ^= low
    return out


@dataclass
class RankedNode:
    """RankedNode (rank.go:21-36) plus the AllocMetric counters."""
    row: int
    node: Optional[Node]
    final_score: float
    scores: List[float] = field(default_factory=list)
    nodes_evaluated: int = 0
    nodes_filtered: int = 0
    nodes_exhausted: int = 0
    new_offset: int = 0
    preempted: List[int] = field(default_factory=list)   # PreemptedAllocs: alloc-table rows
    device_offers: List[int] = field(default_factory=list)   # chosen device group per request
    reserved_cores: List[int] = field(default_factory=list)  # Cpu.ReservedCores of the tasks, ascending

    @classmethod
    def from_c(cls, r: abi.pe_ranked_node, nodes, full_preempted=None):
        """`full_preempted`: the whole PreemptedAllocs list when the record
        carries more than PE_MAX_PREEMPT (pe_preempted_of)."""
        pre = list(full_preempted) if full_preempted is not None else \
            [r.preempted[i] for i in range(min(r.n_preempted, abi.PE_MAX_PREEMPT))]
        return cls(row=r.row, node=nodes[r.row] if (nodes is not None and r.row >= 0) else None,
                   final_score=r.final_score,
                   scores=[r.scores[i] for i in range(r.n_scores)], nodes_evaluated=r.nodes_evaluated,
                   nodes_filtered=r.nodes_filtered, nodes_exhausted=r.nodes_exhausted,
                   new_offset=r.new_offset, preempted=pre,
                   device_offers=[r.device_offer_group[i] for i in range(r.n_device_offers)],
                   reserved_cores=_core_ids(r.reserved_cores))


class _Stack:
    """Stack over a C ABI with a given symbol prefix (engine: 'pe_')."""

    stack_kind = abi.PE_STACK_GENERIC

    def __init__(self, lib, prefix: str, batch: bool = False, config: SchedulerConfig = None,
                 device: int = 0, devices: Optional[Sequence[int]] = None):
        self._lib = lib
        self._p = prefix
        config = config or SchedulerConfig()
        cfg = abi.pe_config()
        cfg.stack_kind = self.stack_kind
        cfg.batch = int(batch)
        cfg.algorithm = abi.PE_ALGO_SPREAD if config.algorithm == "spread" else abi.PE_ALGO_BINPACK
        cfg.memory_oversubscription = int(config.memory_oversubscription)
        cfg.preempt = int(config.preempt_system if self.stack_kind == abi.PE_STACK_SYSTEM
                          else config.preempt_service)
        cfg.device = device
        if devices is not None and len(devices) > 1:   # one handle over several GPUs (pe_config.device_ids)
            if len(devices) > 8:
                raise ValueError("at most 8 devices per handle")
            cfg.device_count = len(devices)
            for k, d in enumerate(devices):
                cfg.device_ids[k] = int(d)
        self._cfg = cfg
        create = getattr(lib, prefix + ("stack_create" if prefix == "pe_" else "create"))
        self._h = create(C.byref(cfg))
        if not self._h:
            err = getattr(lib, prefix + "last_error")(None)
            raise EngineError(-1, (err or b"stack creation failed").decode())
        self.state: Optional[EncodedState] = None
        self.job: Optional[EncodedJob] = None
        self.nodes: List[Node] = []
        self.limit = None

    def close(self):
        if self._h:
            destroy = getattr(self._lib, self._p + ("stack_destroy" if self._p == "pe_" else "destroy"))
            destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != abi.PE_OK:
            msg = getattr(self._lib, self._p + "last_error")(self._h).decode()
            raise (Unsupported if rc == abi.PE_EUNSUPPORTED else EngineError)(rc, msg)

    def _fn(self, name):
        return getattr(self._lib, self._p + name)

    # -- AllocMetric maps (structs.go:9826-10026) ------------------------------
    def EnableMetrics(self, on: bool = True):
        """Collect ClassFiltered / ConstraintFiltered / ClassExhausted /
        DimensionExhausted per Select (before the eval's first Select)."""
        if hasattr(self._lib, self._p + "set_metrics"):
            fn = self._fn("set_metrics")
            fn.restype = C.c_int
            fn.argtypes = [C.c_void_p, C.c_int]
            self._check(fn(self._h, int(on)))

    def LastMetrics(self) -> Dict[str, Dict[str, int]]:
        """The last Select's maps: {"ClassFiltered": {...}, "ConstraintFiltered": {...},
        "ClassExhausted": {...}, "DimensionExhausted": {...}, "ScoreMetaData":
        [(node id, NormScore, {scorer: score}), ...]}."""
        fn = self._fn("last_metrics")
        fn.restype = C.c_int64
        fn.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        need = fn(self._h, None, 0)
        if need < 0:
            self._check(int(need))
        buf = C.create_string_buffer(int(need) + 1)
        fn(self._h, buf, len(buf))
        return parse_metrics(buf.value.decode())

    def LastMetricsBin(self) -> Dict:
        """The last Select's maps from their binary form (pe_last_metrics_bin),
        in LastMetrics' shape: what the Go shim reads without parsing text."""
        lib = self._lib
        lib.pe_last_metrics_bin.restype = C.c_int
        lib.pe_last_metrics_bin.argtypes = [C.c_void_p, C.POINTER(C.POINTER(abi.pe_metric_count)), abi.u32p,
                                            C.POINTER(C.POINTER(abi.pe_metric_score)), abi.u32p]
        c, sc = C.POINTER(abi.pe_metric_count)(), C.POINTER(abi.pe_metric_score)()
        nc, ns = C.c_uint32(0), C.c_uint32(0)
        self._check(lib.pe_last_metrics_bin(self._h, C.byref(c), C.byref(nc), C.byref(sc), C.byref(ns)))
        return decode_metrics(self, c, 0, nc.value, sc, 0, ns.value)

    def MetricString(self, key: int) -> str:
        """pe_metric_string: the text of an AllocMetric key."""
        fn = self._lib.pe_metric_string
        fn.restype = C.c_int64
        fn.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t]
        need = fn(self._h, key, None, 0)
        if need < 0:
            self._check(int(need))
        buf = C.create_string_buffer(int(need) + 1)
        fn(self._h, key, buf, len(buf))
        return buf.value.decode()

    # -- EvalEligibility and iterator state (context.go:190-356) -------------
    def Eligibility(self, changed_only: bool = False) -> Dict:
        """The evaluation's EvalEligibility maps as the reference chain holds
        them: {"job": {class: eligible}, "tgs": {tg name: {class: eligible}},
        "escaped": HasEscaped()} (pe_get_eligibility)."""
        fn = self._fn("get_eligibility")
        n, flags = C.c_uint32(0), C.c_uint32(0)
        self._check(fn(self._h, int(changed_only), None, 0, C.byref(n), C.byref(flags)))
        buf = (abi.pe_class_feas * max(1, n.value))()
        self._check(fn(self._h, int(changed_only), buf, n.value, C.byref(n), C.byref(flags)))
        strs = self.state.interner.strs
        out = {"job": {}, "tgs": {}, "escaped": bool(flags.value & abi.PE_ELIG_ESCAPED)}
        for e in buf[:n.value]:
            cls, ok = strs[e.computed_class], e.status == abi.PE_CLASS_ELIGIBLE
            if e.task_group == abi.PE_NONE:
                out["job"][cls] = ok
            else:
                out["tgs"].setdefault(strs[e.task_group], {})[cls] = ok
        return out

    def PutEligibility(self, elig: Dict):
        """Load EvalEligibility maps ({"job": ..., "tgs": ...}) into this stack's memo."""
        it = self.state.interner
        ents = [(abi.PE_NONE, it.intern(c), ok) for c, ok in elig.get("job", {}).items()]
        for tg, m in elig.get("tgs", {}).items():
            ents += [(it.intern(tg), it.intern(c), ok) for c, ok in m.items()]
        buf = (abi.pe_class_feas * max(1, len(ents)))()
        for k, (tg, c, ok) in enumerate(ents):
            buf[k].task_group, buf[k].computed_class = tg, c
            buf[k].status = abi.PE_CLASS_ELIGIBLE if ok else abi.PE_CLASS_INELIGIBLE
        self._check(self._fn("put_eligibility")(self._h, buf, len(ents)))

    @staticmethod
    def GetClasses(elig: Dict) -> Dict[str, bool]:
        """EvalEligibility.GetClasses (context.go:253-290) over Eligibility()'s maps."""
        out: Dict[str, bool] = {}
        for classes in elig["tgs"].values():
            for cls, ok in classes.items():
                if ok:
                    out[cls] = True
                elif cls not in out:
                    out[cls] = False
        for cls, ok in elig["job"].items():
            if ok:
                out.setdefault(cls, True)
            else:
                out[cls] = False
        return out

    def GetCursor(self):
        """(StaticIterator offset, LimitIterator limit)."""
        off, lim = C.c_uint32(0), C.c_uint32(0)
        self._check(self._fn("get_cursor")(self._h, C.byref(off), C.byref(lim)))
        return off.value, lim.value

    def SetCursor(self, offset: int, limit: int, tg=None):
        """Adopt another chain's cursor and limit; `tg`: the task group it
        selected for (its SpreadIterator.SetTaskGroup ran)."""
        tgi = abi.PE_NONE if tg is None else self._tg_index(tg)
        self._check(self._fn("set_cursor")(self._h, tgi, int(offset), int(limit)))

    # -- scheduler.State snapshot -------------------------------------------
    def SetState(self, nodes: Sequence[Node], allocs: Sequence[Allocation] = ()):
        self.nodes = list(nodes)
        self.state = EncodedState(nodes, allocs, Interner())
        t = self.state.strtab()
        self._check(self._fn("set_state")(self._h, C.byref(t), C.byref(self.state.node_table),
                                          C.byref(self.state.alloc_table)))
        return self.state

    def SetStateColumnar(self, cs):
        """Snapshot from a synth_columnar.ColumnarState (no per-node Python objects)."""
        self.nodes = None
        self.state = cs
        t = cs.strtab()
        self._check(self._fn("set_state")(self._h, C.byref(t), C.byref(cs.node_table), C.byref(cs.alloc_table)))
        return cs

    def UpdateAllocs(self, allocs: Sequence[Allocation], index: Optional[Sequence[int]] = None):
        """State delta without a node reload (pe_update_allocs): allocs[i]
        replaces snapshot alloc index[i] (None / -1: appended)."""
        fn = self._fn("update_allocs")
        fn.restype = C.c_int
        fn.argtypes = [C.c_void_p, C.POINTER(abi.pe_strtab), C.POINTER(abi.pe_alloc_table), abi.u32p]
        at = self.state.encode_alloc_table(allocs)
        idx = np.asarray([abi.PE_NONE if (index is None or index[i] is None or index[i] < 0) else index[i]
                          for i in range(len(allocs))] or [0], dtype=np.uint32)
        t = self.state.strtab()
        self._check(fn(self._h, C.byref(t), C.byref(at), idx.ctypes.data_as(abi.u32p)))
        self._job = None

    def UpdateNodes(self, nodes: Sequence[Node], index: Optional[Sequence[int]] = None):
        """Node upserts without a reload (pe_update_nodes): nodes[i] replaces
        snapshot row index[i] (None / -1: appended)."""
        fn = self._fn("update_nodes")
        fn.restype = C.c_int
        fn.argtypes = [C.c_void_p, C.POINTER(abi.pe_strtab), C.POINTER(abi.pe_node_table), abi.u32p]
        nt, idx = self.state.update_nodes(nodes, index)
        if self.nodes is not None:
            self.nodes = list(self.state.nodes)
        t = self.state.strtab()
        self._check(fn(self._h, C.byref(t), C.byref(nt), idx.ctypes.data_as(abi.u32p)))
        self._job = None

    def ResetPlan(self):
        """New evaluation on the resident snapshot (fresh EvalContext)."""
        self._check(self._fn("reset_plan")(self._h))

    def row(self, node_or_id) -> int:
        nid = node_or_id if isinstance(node_or_id, str) else node_or_id.id
        return self.state.row_of[nid]

    # -- Stack interface -------------------------------------------------------
    def SetJob(self, job: Job):
        self.job = EncodedJob(job, self.state.interner)
        self._job = job
        t = self.job.strtab()
        self._check(self._fn("set_job")(self._h, C.byref(t), C.byref(self.job.job)))

    def SetNodes(self, nodes_in_visit_order) -> int:
        """`nodes_in_visit_order`: Node objects / IDs / rows, already shuffled."""
        if isinstance(nodes_in_visit_order, np.ndarray) and nodes_in_visit_order.dtype.kind in "iu":
            rows = np.ascontiguousarray(nodes_in_visit_order, dtype=np.uint32)
        else:
            rows = np.asarray([x if isinstance(x, (int, np.integer)) else self.row(x)
                               for x in nodes_in_visit_order], dtype=np.uint32)
        self._visit = rows
        lim = C.c_uint32(0)
        self._check(self._fn("set_nodes")(self._h, rows.ctypes.data_as(abi.u32p), len(rows), C.byref(lim)))
        self.limit = lim.value
        return self.limit

    def _tg_index(self, tg):
        if isinstance(tg, int):
            return tg
        for i, g in enumerate(self._job.task_groups):
            if g is tg or g.name == tg:
                return i
        raise KeyError(tg)

    def Select(self, tg, options: SelectOptions = None) -> Optional[RankedNode]:
        opts = abi.pe_select_options()
        keep = []
        if options is not None:
            if options.penalty_node_ids:
                pen = np.asarray([self.row(x) for x in options.penalty_node_ids], dtype=np.uint32)
                keep.append(pen)
                opts.penalty_rows, opts.penalty_count = pen.ctypes.data_as(abi.u32p), len(pen)
            if options.preferred_nodes:
                pref = np.asarray([self.row(x) for x in options.preferred_nodes], dtype=np.uint32)
                keep.append(pref)
                opts.preferred_rows, opts.preferred_count = pref.ctypes.data_as(abi.u32p), len(pref)
            opts.preempt = int(options.preempt)
        out = abi.pe_ranked_node()
        self._check(self._fn("select")(self._h, self._tg_index(tg), C.byref(opts), C.byref(out)))
        r = RankedNode.from_c(out, self.nodes, self._full_preempted(0, out))
        return r if r.row >= 0 else None

    def _full_preempted(self, record, r):
        """PreemptedAllocs of record `record` of the last call when the record
        holds more than PE_MAX_PREEMPT inline (else None)."""
        if r.n_preempted <= abi.PE_MAX_PREEMPT:
            return None
        buf = (C.c_uint32 * r.n_preempted)()
        n = self._fn("preempted_of")(self._h, record, buf, r.n_preempted)
        if n != r.n_preempted:
            raise RuntimeError("preempted_of(%d) returned %d for %d allocs" % (record, n, r.n_preempted))
        return list(buf)

    def SelectRaw(self, tg, options: SelectOptions = None) -> RankedNode:
        """Select, but also returns the metrics when no node was found."""
        out = abi.pe_ranked_node()
        opts = abi.pe_select_options()
        if options is not None:
            opts.preempt = int(options.preempt)
        self._check(self._fn("select")(self._h, self._tg_index(tg), C.byref(opts), C.byref(out)))
        return RankedNode.from_c(out, self.nodes, self._full_preempted(0, out))

    def Commit(self, tg, node_or_row, preempted: Sequence[int] = ()):
        """Plan.AppendAlloc (+ AppendPreemptedAlloc of `preempted` alloc-table rows)."""
        row = node_or_row if isinstance(node_or_row, (int, np.integer)) else self.row(node_or_row)
        if len(preempted):
            pre = np.asarray(preempted, dtype=np.uint32)
            self._check(self._fn("commit_preempt")(self._h, self._tg_index(tg), int(row),
                                                   pre.ctypes.data_as(abi.u32p), len(pre)))
        else:
            self._check(self._fn("commit")(self._h, self._tg_index(tg), int(row)))

    def StopAllocs(self, allocs: Sequence[int]):
        """Plan.AppendStoppedAlloc of snapshot allocs (alloc-table rows)."""
        a = np.ascontiguousarray(np.asarray(list(allocs) or [0], dtype=np.uint32))
        self._check(self._fn("plan_stop")(self._h, a.ctypes.data_as(abi.u32p), len(allocs)))

    def PopUpdate(self, alloc: int):
        """Plan.PopUpdate of a snapshot alloc (alloc-table row)."""
        self._check(self._fn("plan_pop_update")(self._h, int(alloc)))

    def Place(self, tg, count: int) -> List[RankedNode]:
        out = (abi.pe_ranked_node * max(1, count))()
        placed = C.c_uint32(0)
        self._check(self._fn("place")(self._h, self._tg_index(tg), count, out, C.byref(placed)))
        n = min(count, placed.value + 1)
        return [RankedNode.from_c(out[i], self.nodes, self._full_preempted(i, out[i])) for i in range(n)]

    def PlaceArrays(self, tg, count: int):
        """Fused count loop returning (rows, final_scores, placed, records) as numpy
        arrays. The record buffer is reused across calls with the same count."""
        cache = getattr(self, "_place_buf", None)
        if cache is None or cache[0] != count:
            out = (abi.pe_ranked_node * max(1, count))()
            cache = (count, out, np.ctypeslib.as_array(out), C.c_uint32(0))
            self._place_buf = cache
        _, out, arr, placed = cache
        self._check(self._fn("place")(self._h, self._tg_index(tg), count, out, C.byref(placed)))
        return arr["row"].copy(), arr["final_score"].copy(), placed.value, arr

    def SystemPlaceView(self, tg):
        """SystemPlace with the results left in the engine's page-locked
        staging (pe_system_place with null arrays + pe_system_results): numpy
        views valid until the next SystemPlace on this stack, no copy."""
        placed = C.c_uint32(0)
        self._check(self._fn("system_place")(self._h, self._tg_index(tg), None, None, C.byref(placed)))
        lib = self._lib
        lib.pe_system_results.restype = C.c_int
        lib.pe_system_results.argtypes = [C.c_void_p, C.POINTER(abi.f64p), C.POINTER(abi.u8p), abi.u32p]
        sc, st, n = abi.f64p(), abi.u8p(), C.c_uint32(0)
        self._check(lib.pe_system_results(self._h, C.byref(sc), C.byref(st), C.byref(n)))
        if n.value == 0:
            return np.empty(0), np.empty(0, dtype=np.uint8), placed.value
        return (np.ctypeslib.as_array(sc, shape=(n.value,)), np.ctypeslib.as_array(st, shape=(n.value,)),
                placed.value)

    def SystemPlace(self, tg):
        n = len(self._visit)
        score = np.empty(max(1, n), dtype=np.float64)
        status = np.empty(max(1, n), dtype=np.uint8)
        placed = C.c_uint32(0)
        self._check(self._fn("system_place")(self._h, self._tg_index(tg), score.ctypes.data_as(abi.f64p),
                                             status.ctypes.data_as(abi.u8p), C.byref(placed)))
        return score[:n], status[:n], placed.value


class GenericStack(_Stack):
    """NewGenericStack (stack.go:336-431) on the MI355X engine."""
    stack_kind = abi.PE_STACK_GENERIC

    def __init__(self, batch: bool = False, config: SchedulerConfig = None, device: int = 0,
                 devices: Optional[Sequence[int]] = None):
        super().__init__(load_engine(), "pe_", batch, config, device, devices)

    def StageOrders(self, orders: np.ndarray):
        """Stage E visit orders (E x n rows, each a shuffled SetNodes list) in HBM."""
        o = np.ascontiguousarray(np.asarray(orders, dtype=np.uint32))
        if o.ndim != 2:
            raise ValueError("orders must be 2-D (evals x nodes)")
        self._check(self._lib.pe_stage_orders(self._h, o.ctypes.data_as(abi.u32p), o.shape[0], o.shape[1]))
        self._staged = o.shape[0]

    _PLACEMENT = np.dtype([("row", "<i4"), ("nodes_evaluated", "<u4"), ("final_score", "<f8")])

    def PlaceBatch(self, tg, count: int, copy: bool = True):
        """Independent evaluations over the staged orders; returns (rows, scores, evaluated, placed).

        copy=False returns views of the engine's page-locked result buffer
        (valid until the next PlaceBatch) instead of copies."""
        self._check(self._lib.pe_place_batch(self._h, self._tg_index(tg), count, None, None))
        res = C.POINTER(abi.pe_placement)()
        status = abi.u32p()
        n_evals, cnt = C.c_uint32(0), C.c_uint32(0)
        self._check(self._lib.pe_batch_results(self._h, C.byref(res), C.byref(status), C.byref(n_evals),
                                               C.byref(cnt)))
        E = n_evals.value
        total = E * count
        if total:
            raw = np.ctypeslib.as_array(C.cast(res, C.POINTER(C.c_uint8)), shape=(total * 16,))
            out = raw.view(self._PLACEMENT).reshape(E, count)
            st = np.ctypeslib.as_array(status, shape=(2 * E,))
            placed = st[0::2]
        else:
            out = np.zeros((E, count), dtype=self._PLACEMENT)
            placed = np.zeros(E, dtype=np.uint32)
        if copy:
            out = out.copy()
            placed = placed.copy()
        return out["row"], out["final_score"], out["nodes_evaluated"], placed

    def SelectShard(self, tg, row_begin: int, row_end: int) -> bytes:
        """This GPU's part of a full-pass Select: the 80-byte record of snapshot
        rows [row_begin, row_end) (pe_select_shard)."""
        rec = abi.pe_shard_rec()
        self._check(self._lib.pe_select_shard(self._h, self._tg_index(tg), row_begin, row_end, C.byref(rec)))
        return bytes(rec.bytes)

    def SelectMerge(self, tg, recs) -> RankedNode:
        """Resolve the Select from every shard's record (pe_select_merge)."""
        arr = (abi.pe_shard_rec * max(1, len(recs)))()
        for i, r in enumerate(recs):
            C.memmove(arr[i].bytes, bytes(r), 80)
        out = abi.pe_ranked_node()
        self._check(self._lib.pe_select_merge(self._h, self._tg_index(tg), arr, len(recs), C.byref(out)))
        return RankedNode.from_c(out, self.nodes)

    def CommInit(self, nranks: int, rank: int, unique_id: bytes):
        """Join the RCCL communicator of `nranks` engines (pe_comm_init); every
        rank passes the same 128-byte id (comm_unique_id on one rank)."""
        buf = np.frombuffer(bytes(unique_id), dtype=np.uint8).copy()
        self._check(self._lib.pe_comm_init(self._h, nranks, rank, buf.ctypes.data_as(abi.u8p)))

    def CommInitHost(self, nranks: int, rank: int, all_gather):
        """Join `nranks` engines over a caller transport (pe_comm_init_host):
        all_gather(record: bytes) -> list of nranks records in rank order, called
        once per placement of PlaceSharded (e.g. torch.distributed over gloo)."""
        def exchange(_ctx, send, recv, nbytes):
            try:
                recs = all_gather(C.string_at(send, nbytes))
                if len(recs) != nranks or any(len(r) != nbytes for r in recs):
                    return 2
                C.memmove(recv, b"".join(recs), nbytes * nranks)
                return 0
            except Exception:   # noqa: BLE001 - reported to the engine as a failed exchange
                return 1
        self._xfn = abi.pe_exchange_fn(exchange)   # kept alive with the handle
        self._check(self._lib.pe_comm_init_host(self._h, nranks, rank, self._xfn, None))

    def PlaceSharded(self, tg, count: int, row_begin: int, row_end: int) -> List[RankedNode]:
        """The full-pass count loop over the communicator's ranks, this rank
        sweeping snapshot rows [row_begin, row_end) (pe_place_sharded); every
        rank returns the same records."""
        out = (abi.pe_ranked_node * max(1, count))()
        placed = C.c_uint32(0)
        self._check(self._lib.pe_place_sharded(self._h, self._tg_index(tg), count, row_begin, row_end, out,
                                               C.byref(placed)))
        n = min(count, placed.value + 1)
        return [RankedNode.from_c(out[i], self.nodes) for i in range(n)]

    def last_exchange_us(self) -> float:
        """Device time of the all-gather in the last PlaceSharded (us, mean over every placement)."""
        return self._lib.pe_last_exchange_us(self._h)

    def last_exchange_stats(self):
        """(mean, min, max) us of the last PlaceSharded's all-gathers and the placements timed."""
        out = (C.c_double * 4)()
        self._lib.pe_last_exchange_stats(C.c_void_p(self._h), out)
        return float(out[0]), float(out[1]), float(out[2]), int(out[3])

    def SpeculationStats(self):
        """(runs, Selects answered from records, rollbacks, records computed) of
        the speculative count loop behind Select / Commit (pe_speculation_stats)."""
        buf = (C.c_uint64 * 4)()
        self._check(self._lib.pe_speculation_stats(self._h, buf))
        return tuple(int(x) for x in buf)

    def last_phase_ms(self):
        """[host prep, kernel, D2H copy, total] of the last PlaceBatch, ms."""
        buf = (C.c_double * 4)()
        self._lib.pe_last_phase_ms(self._h, C.cast(buf, abi.f64p))
        return list(buf)

    def last_kernel_ms(self) -> float:
        return self._lib.pe_last_kernel_ms(self._h)

    def last_sweep_bytes(self) -> int:
        """Algorithmic bytes per node of the last full-scan sweep Select."""
        return self._lib.pe_last_sweep_bytes(self._h)

    def SetKernelSplit(self, on: bool = True):
        """Record HIP events between the windowed chain's kernels (measurement aid)."""
        self._check(self._lib.pe_set_kernel_split(self._h, 1 if on else 0))

    def last_kernel_split(self):
        """{k_base, k_chain, k_emit, k_emit_writeback} device ms of the last chain launch."""
        buf = (C.c_double * 4)()
        self._check(self._lib.pe_last_kernel_split(self._h, C.cast(buf, abi.f64p)))
        return dict(zip(("k_base", "k_chain", "k_emit", "k_emit_writeback"), list(buf)))


def comm_unique_id() -> bytes:
    """ncclGetUniqueId through the engine (pe_comm_unique_id): 128 bytes that
    rank 0 hands to every rank's CommInit."""
    buf = np.zeros(128, dtype=np.uint8)
    rc = load_engine().pe_comm_unique_id(buf.ctypes.data_as(abi.u8p), 128)
    if rc:
        raise RuntimeError("pe_comm_unique_id failed (%d)" % rc)
    return buf.tobytes()


class SystemStack(_Stack):
    """NewSystemStack (stack.go:207-283) on the MI355X engine."""
    stack_kind = abi.PE_STACK_SYSTEM

    def __init__(self, sysbatch: bool = False, config: SchedulerConfig = None, device: int = 0,
                 devices: Optional[Sequence[int]] = None):
        super().__init__(load_engine(), "pe_", False, config, device, devices)

    def last_kernel_ms(self) -> float:
        return self._lib.pe_last_kernel_ms(self._h)
