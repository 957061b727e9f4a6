"""Caller-side harness (bench / tests only): runs tools/libdropin.so, the Go
caller's Select -> Commit loop in C (generic_sched.go:472-652, 773-816),
against an engine GenericStack or an OracleGenericStack that already holds a
snapshot (SetState). Evaluations: ResetPlan, SetJob, SetNodes(order), then
count x (Select [, Select Preempt] , Commit)."""
import ctypes as C
import os
import subprocess

import numpy as np

from nomad_amd import abi
from nomad_amd.encode import EncodedJob

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libdropin.so")
_lib = None


class dropin_api(C.Structure):
    _fields_ = [(name, C.c_void_p) for name in
                ("reset_plan", "set_job", "set_nodes", "select", "commit", "commit_preempt", "preempted_of",
                 "spec_view_get", "system_view_get", "last_metrics", "last_metrics_bin")]


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", HERE])
        lib = C.CDLL(LIB)
        lib.dropin_phase_seconds.restype = None
        lib.dropin_phase_seconds.argtypes = [C.POINTER(C.c_double), C.c_int]
        lib.dropin_evals.restype = C.c_int
        lib.dropin_evals.argtypes = [C.POINTER(dropin_api), C.c_void_p, C.POINTER(abi.pe_strtab),
                                     C.POINTER(abi.pe_job), abi.u32p, C.c_uint32, C.c_uint32, C.c_uint32,
                                     C.c_uint32, C.c_int, C.c_uint32, C.c_double, abi.i32p,
                                     C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
        lib.dropin_use_view.restype = None
        lib.dropin_use_view.argtypes = [C.c_int]
        lib.dropin_view_served.restype = C.c_uint64
        lib.dropin_view_served.argtypes = [C.c_int]
        lib.dropin_system_phases.restype = None
        lib.dropin_system_phases.argtypes = [C.POINTER(C.c_double), C.c_int]
        lib.dropin_use_metrics.restype = None
        lib.dropin_use_metrics.argtypes = [C.c_int]
        lib.dropin_metric_bytes.restype = C.c_uint64
        lib.dropin_metric_bytes.argtypes = [C.c_int]
        lib.dropin_system.restype = C.c_int
        lib.dropin_system.argtypes = [C.POINTER(dropin_api), C.c_void_p, C.c_uint32, abi.u32p, C.c_uint32,
                                      abi.u8p, abi.f64p, abi.u32p, C.c_void_p, C.POINTER(C.c_double)]
        _lib = lib
    return _lib


def _api(stack):
    lib, p = stack._lib, stack._p
    a = dropin_api()
    for name, _ in dropin_api._fields_:
        fn = getattr(lib, p + name, None)   # the oracle has no served-Select view
        setattr(a, name, C.cast(fn, C.c_void_p).value if fn is not None else None)
    return a


def use_view(on):
    """Whether the C loop answers plain Select / Commit pairs from the
    engine's served-Select view (the Go shim's shape) or crosses every time."""
    load().dropin_use_view(1 if on else 0)


def use_metrics(on):
    """Whether the C loop copies out every Select's AllocMetric maps (the
    stack must have them on: EnableMetrics), as the shim fills
    Allocation.Metrics."""
    load().dropin_use_metrics(1 if on else 0)


def metric_bytes(reset=False):
    return int(load().dropin_metric_bytes(1 if reset else 0))


def view_served(reset=False):
    return int(load().dropin_view_served(1 if reset else 0))


def prepare(stack, job):
    """Encode `job` for `stack` once (what a cgo shim does when the job comes
    in) and return run(orders, count, tg=0, preempt=False, n_evals=None,
    max_seconds=0.0): sequential evaluations through the C loop. orders: (k, n)
    visit orders, evaluation e uses orders[e % k]. run returns (placements,
    evals, selects, seconds, rows of the last evaluation)."""
    lib = load()
    enc = EncodedJob(job, stack.state.interner)
    tab = enc.strtab()
    api = _api(stack)
    out = (C.c_uint64 * 3)()
    secs = C.c_double(0.0)

    def run(orders, count, tg=0, preempt=False, n_evals=None, max_seconds=0.0):
        o = np.ascontiguousarray(np.atleast_2d(np.asarray(orders, dtype=np.uint32)))
        rows = np.full(max(1, count), -1, dtype=np.int32)
        ne = o.shape[0] if n_evals is None else n_evals
        rc = lib.dropin_evals(C.byref(api), stack._h, C.byref(tab), C.byref(enc.job), o.ctypes.data_as(abi.u32p),
                              o.shape[0], o.shape[1], tg, count, int(preempt), ne, max_seconds,
                              rows.ctypes.data_as(abi.i32p), out, C.byref(secs))
        stack._check(rc)
        stack._job = job
        return int(out[0]), int(out[1]), int(out[2]), secs.value, rows[:count]
    run.keep = (enc, tab, api)   # the C structs point into these
    return run


def run(stack, job, orders, count, tg=0, preempt=False, n_evals=None, max_seconds=0.0):
    """Sequential evaluations of `job` through the C loop (see prepare)."""
    return prepare(stack, job)(orders, count, tg=tg, preempt=preempt, n_evals=n_evals, max_seconds=max_seconds)


PHASES = ("reset_plan", "set_job", "set_nodes", "first_select", "loop")


def phase_seconds(reset=True):
    """Wall seconds per caller phase summed over dropin_evals calls."""
    out = (C.c_double * 5)()
    load().dropin_phase_seconds(out, int(reset))
    return dict(zip(PHASES, list(out)))


def system_phases(reset=True):
    """Seconds of dropin_system's parts summed since the last reset: triples
    that crossed into C, the whole loop, the final flush."""
    out = (C.c_double * 3)()
    load().dropin_system_phases(out, int(reset))
    return {"crossing": out[0], "loop": out[1], "flush": out[2]}


def system_loop(stack, tg, rows, flush=True):
    """SystemScheduler.computePlacements' per-node loop through the C harness
    (SetNodes([node]) + Select + Commit for every node of `rows`) on a
    SystemStack that holds the snapshot and the job. Returns (status, score,
    placed, seconds); `flush` times pe_flush (queued commits into HBM) too."""
    lib = load()
    r = np.ascontiguousarray(np.asarray(rows, dtype=np.uint32))
    st = np.zeros(max(1, len(r)), dtype=np.uint8)
    sc = np.zeros(max(1, len(r)), dtype=np.float64)
    placed, secs = C.c_uint32(0), C.c_double(0.0)
    fl = C.cast(getattr(stack._lib, stack._p + "flush"), C.c_void_p).value \
        if flush and hasattr(stack._lib, stack._p + "flush") else None
    api = _api(stack)
    rc = lib.dropin_system(C.byref(api), stack._h, tg, r.ctypes.data_as(abi.u32p), len(r),
                           st.ctypes.data_as(abi.u8p), sc.ctypes.data_as(abi.f64p), C.byref(placed), fl,
                           C.byref(secs))
    stack._check(rc)
    return st[:len(r)], sc[:len(r)], placed.value, secs.value
