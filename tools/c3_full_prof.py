"""C3 bench shape through pe_place (k_fullpass_lds): per-phase clocks of the
loop (PE_FULL_PROF=1 prints them on stderr) and the wall per placement."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nomad_amd import synth  # noqa: E402
from nomad_amd.stack import GenericStack  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
nodes, allocs = synth.cluster_c3(n, seed=7)
job = synth.job_c3(1000)
perm = synth.shuffle(n, 17)
st = GenericStack()
st.SetState(nodes, allocs)
for i in range(3):
    st.ResetPlan()
    st.SetJob(job)
    st.SetNodes(perm)
    t0 = time.perf_counter()
    rows, _, placed, _ = st.PlaceArrays(0, 1000)
    dt = time.perf_counter() - t0
    print("pe_place %d placements: wall %.1f us/placement, kernel %.2f us/placement"
          % (placed, dt / placed * 1e6, st.last_kernel_ms() / placed * 1e3), flush=True)
