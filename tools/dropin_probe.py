"""Probe (GPU box): where one drop-in evaluation's time goes. Runs the C2
caller loop (tools/libdropin.so) on a 10k-node cluster and prints the per-phase
wall time per evaluation (reset_plan, set_job, set_nodes, first Select = the
speculative count loop, rest of the Select/Commit loop), then one k_chain
step profile (PE_CHAIN_PROF) and one pe_place profile (PE_PLACE_PROF).

usage: python tools/dropin_probe.py [nodes] [count] [evals]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from nomad_amd import synth  # noqa: E402
from nomad_amd.stack import GenericStack  # noqa: E402
from tools import dropin  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    count = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    evals = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    nodes, allocs = synth.cluster_c2(n, seed=42)
    job = synth.job_c2(count)
    orders = np.stack([synth.shuffle(n, 1000 + e) for e in range(32)])
    if os.environ.get("PROBE_NO_SPIN"):
        os.environ["PE_SPIN_WAIT"] = "0"
    st = GenericStack()
    os.environ.pop("PE_SPIN_WAIT", None)
    st.SetState(nodes, allocs)
    run = dropin.prepare(st, job)
    run(orders, count, n_evals=5)
    dropin.phase_seconds(reset=True)
    t0 = time.perf_counter()
    placed, ne, _, secs, _ = run(orders, count, n_evals=evals)
    wall = time.perf_counter() - t0
    ph = dropin.phase_seconds(reset=True)
    print("evals %d placed %d: %.1f us per eval (C loop %.1f us), %.3g placements/s"
          % (ne, placed, wall / ne * 1e6, secs / ne * 1e6, placed / wall))
    for k, v in ph.items():
        print("  %-13s %8.1f us per eval" % (k, v / ne * 1e6))
    print("  speculation stats", st.SpeculationStats())
    # single entry points, each timed alone (ctypes overhead ~1 us included)
    lib = st._lib
    h = st._h
    enc, tab, _ = run.keep
    import ctypes as C
    rows = np.ascontiguousarray(orders[0])
    lim = C.c_uint32(0)
    reps = 200

    def timed(name, fn):
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        print("  %-28s %7.1f us" % (name, (time.perf_counter() - t) / reps * 1e6))
    timed("pe_reset_plan", lambda: lib.pe_reset_plan(h))
    timed("pe_reset_plan + set_job", lambda: (lib.pe_reset_plan(h), lib.pe_set_job(h, C.byref(tab), C.byref(enc.job))))
    timed("pe_set_nodes", lambda: lib.pe_set_nodes(h, rows.ctypes.data_as(C.POINTER(C.c_uint32)), len(rows),
                                                   C.byref(lim)))
    timed("pe_abi_version (ctypes floor)", lambda: lib.pe_abi_version())

    def spin_us(us):
        t = time.perf_counter()
        while (time.perf_counter() - t) * 1e6 < us:
            pass
    for gap in (20, 100, 200, 1000):
        tot = 0.0
        for _ in range(100):
            spin_us(gap)
            t = time.perf_counter()
            lib.pe_reset_plan(h)
            tot += time.perf_counter() - t
        print("  pe_reset_plan after %4d us idle  %7.1f us" % (gap, tot / 100 * 1e6))
    st.close()
    os.environ["PE_CHAIN_PROF"] = "1"
    os.environ["PE_PLACE_PROF"] = "1"
    st2 = GenericStack()
    st2.SetState(nodes, allocs)
    for _ in range(3):
        st2.ResetPlan()
        st2.SetJob(job)
        st2.SetNodes(orders[0])
        st2.PlaceArrays(0, count)
        print("  PlaceArrays kernel ms %.4f" % st2.last_kernel_ms(), flush=True)
    st2.close()


if __name__ == "__main__":
    main()
