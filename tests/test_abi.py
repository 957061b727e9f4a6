"""C-ABI boundary checks (CPU): the library loads, exports every entry point
include/nomad_pe.h declares, its struct layouts match the ctypes mirror, and it
fails loudly (no CPU fallback) when no HIP device is present."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from nomad_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nomad_pe.h")
LIB = os.path.join(ROOT, "nomad_amd", "libnomadpe.so")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^[a-z_0-9 \*]+?\b(pe_[a-z_0-9]+)\s*\(", text, re.M)))


def test_every_declared_symbol_is_exported():
    lib = C.CDLL(LIB)
    names = declared_functions()
    assert "pe_select" in names and "pe_place_batch" in names
    for name in names:
        assert hasattr(lib, name), name
    assert set(abi.ENGINE_SYMBOLS) <= set(names)
    assert set(abi.PLANNER_SYMBOLS) <= set(names)


def test_abi_version():
    lib = C.CDLL(LIB)
    lib.pe_abi_version.restype = C.c_uint32
    assert lib.pe_abi_version() == 9


STRUCTS = ["pe_strtab", "pe_attr", "pe_node_table", "pe_alloc_table", "pe_constraint", "pe_affinity",
           "pe_spread_target", "pe_spread", "pe_device_request", "pe_task", "pe_task_group", "pe_job",
           "pe_config", "pe_select_options", "pe_ranked_node", "pe_placement", "pe_class_feas",
           "pe_plan_node_table", "pe_plan_alloc_table", "pe_plan"]


def test_struct_layouts_match_ctypes():
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"%s\"\nint main(void){\n" % HEADER
    for s in STRUCTS:
        src += '  printf("%s %%zu\\n", sizeof(%s));\n' % (s, s)
    src += "  return 0;\n}\n"
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "sz.c")
        exe = os.path.join(d, "sz")
        open(c, "w").write(src)
        subprocess.check_call(["gcc", "-o", exe, c])
        out = subprocess.check_output([exe]).decode().split("\n")
    sizes = dict(line.split() for line in out if line)
    for s in STRUCTS:
        assert int(sizes[s]) == C.sizeof(getattr(abi, s)), s


def test_engine_fails_loudly_without_gpu():
    lib = C.CDLL(LIB)
    lib.pe_stack_create.restype = C.c_void_p
    lib.pe_stack_create.argtypes = [C.POINTER(abi.pe_config)]
    lib.pe_last_error.restype = C.c_char_p
    lib.pe_last_error.argtypes = [C.c_void_p]
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    cfg = abi.pe_config()
    h = lib.pe_stack_create(C.byref(cfg))
    assert not h
    assert b"no HIP device" in lib.pe_last_error(None)


def test_planner_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from nomad_amd.plan import Planner, PlannerError
    with pytest.raises(PlannerError):
        Planner()
