"""ORACLE — test infrastructure only.

Python binding of oracle/liboracle.so, the CPU restatement of the reference
placement stack (oracle/oracle.cpp). Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg import this module; the product (nomad_amd/) never
does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from nomad_amd import abi
from nomad_amd.stack import _Stack
from nomad_amd.structs import SchedulerConfig

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
_lib = None


def build(native: bool = False):
    env = dict(os.environ)
    if native:
        env["CXXFLAGS"] = ("-O3 -march=native -std=c++17 -fPIC -ffp-contract=off -Wall -Wextra "
                           "-Wno-unused-parameter -Wno-unused-function")
    subprocess.check_call(["make", "-s", "-C", HERE] + (["-B"] if native else []), env=env)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        abi.bind(lib, "oracle_", "oracle_create", "oracle_destroy", "oracle_last_error")
        lib.oracle_full_pass.restype = C.c_int
        lib.oracle_full_pass.argtypes = [C.c_void_p, C.c_uint32, abi.u8p, abi.f64p, C.POINTER(abi.pe_ranked_node)]
        lib.oracle_go_pow.restype = C.c_double
        lib.oracle_go_pow.argtypes = [C.c_double, C.c_double]
        lib.oracle_go_exp.restype = C.c_double
        lib.oracle_go_exp.argtypes = [C.c_double]
        lib.oracle_go_log.restype = C.c_double
        lib.oracle_go_log.argtypes = [C.c_double]
        lib.oracle_score_fit.restype = C.c_double
        lib.oracle_score_fit.argtypes = [C.c_int] + [C.c_int64] * 6
        lib.oracle_check_constraint.restype = C.c_int
        lib.oracle_check_constraint.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_char_p, C.c_int]
        lib.oracle_limit_iter.restype = C.c_int
        lib.oracle_limit_iter.argtypes = [abi.f64p, C.c_int, C.c_int, C.c_double, C.c_int,
                                          abi.i32p, abi.i32p, abi.i32p]
        _lib = lib
    return _lib


class OracleGenericStack(_Stack):
    stack_kind = abi.PE_STACK_GENERIC

    def __init__(self, batch: bool = False, config: SchedulerConfig = None):
        super().__init__(load(), "oracle_", batch, config, 0)


class OracleSystemStack(_Stack):
    stack_kind = abi.PE_STACK_SYSTEM

    def __init__(self, sysbatch: bool = False, config: SchedulerConfig = None):
        super().__init__(load(), "oracle_", False, config, 0)


def go_pow(x, y):
    return load().oracle_go_pow(x, y)


def score_fit(algo, cpu, mem, rcpu, rmem, ucpu, umem):
    return load().oracle_score_fit(algo, cpu, mem, rcpu, rmem, ucpu, umem)


def check_constraint(op, l, r):
    """l / r: a str (found), None (nil: unknown ${...}) or ('', False) style tuple (missing attr)."""
    def enc(v):
        if v is None:
            return None, 0
        if isinstance(v, tuple):
            return v[0].encode(), 2
        return str(v).encode(), 1
    lv, ls = enc(l)
    rv, rs = enc(r)
    return bool(load().oracle_check_constraint(op.encode(), lv, ls, rv, rs))


def limit_iter(scores, limit, threshold=0.0, max_skip=3):
    s = np.ascontiguousarray(np.asarray(scores, dtype=np.float64))
    order = np.zeros(max(1, len(s)), dtype=np.int32)
    w, p = C.c_int32(0), C.c_int32(0)
    k = load().oracle_limit_iter(s.ctypes.data_as(abi.f64p), len(s), limit, threshold, max_skip,
                                 order.ctypes.data_as(abi.i32p), C.byref(w), C.byref(p))
    return list(order[:k]), w.value, p.value


class _PlannerAdapter:
    """pe_planner_* names over liboracle's oracle_planner_* (plan_oracle.cpp)."""

    def __init__(self, lib):
        H = C.c_void_p
        sigs = [("create", C.c_void_p, []), ("destroy", None, [H]),
                ("set_state", C.c_int, [H, C.POINTER(abi.pe_strtab), C.POINTER(abi.pe_plan_node_table),
                                        C.POINTER(abi.pe_plan_alloc_table)]),
                ("evaluate", C.c_int, [H, C.POINTER(abi.pe_strtab), C.POINTER(abi.pe_plan), abi.u8p, abi.u32p]),
                ("commit", C.c_int, [H, C.POINTER(abi.pe_strtab), C.POINTER(abi.pe_plan), abi.u8p])]
        for name, res, args in sigs:
            fn = getattr(lib, "oracle_planner_" + name)
            fn.restype = res
            fn.argtypes = args
            setattr(self, "pe_planner_" + name, fn)

    @staticmethod
    def pe_planner_last_error(h):
        return b"oracle planner"


def OraclePlanner():
    """nomad_amd.plan.Planner's interface (set_state / encode / evaluate /
    evaluate_plan_placements / apply) on the C++ restatement: the same
    encoding of the same plans, evaluated on one CPU core."""
    from nomad_amd.plan import Interner, Planner

    class _OraclePlanner(Planner):
        def __init__(self):
            self.lib = _PlannerAdapter(load())
            self.h = self.lib.pe_planner_create()
            self.nodes, self.row_of, self.allocs, self.alloc_index = [], {}, [], {}
            self.interner = Interner()

        def close(self):
            if getattr(self, "h", None):
                self.lib.pe_planner_destroy(self.h)
                self.h = None

        def kernel_ms(self):
            return 0.0

        def last_bytes(self):
            return 0

    return _OraclePlanner()
