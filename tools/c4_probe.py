"""C4 host-overhead probe: system job on 100k nodes, SetNodes + SystemPlace
timed separately from Python (run with PE_API_PROF=1 for the engine's host
steps, printed when the stack closes)."""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from nomad_amd import synth, synth_columnar  # noqa: E402
from nomad_amd.stack import SystemStack  # noqa: E402

n = 100000
cs = synth_columnar.ColumnarState(n, seed=11, kind="c4", prefill=0.05)
job = synth.mock_system_job()
rows = np.random.Generator(np.random.PCG64(5)).permutation(n).astype(np.uint32)
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 12
st = SystemStack()
st.SetStateColumnar(cs)
walls = []
for i in range(iters):
    view = i >= min(6, iters // 2)   # the zero-copy results (SystemPlaceView) for the second half
    st.ResetPlan()
    st.SetJob(job)
    t0 = time.perf_counter()
    st.SetNodes(rows)
    t1 = time.perf_counter()
    _, _, placed = st.SystemPlaceView(0) if view else st.SystemPlace(0)
    t2 = time.perf_counter()
    if view:
        walls.append((t2 - t0) * 1e6)
    if iters <= 12:
        print("iter %d%s: SetNodes %.1f us, SystemPlace %.1f us (kernel %.1f us), placed %d"
              % (i, " view" if view else "", (t1 - t0) * 1e6, (t2 - t1) * 1e6, st.last_kernel_ms() * 1e3, placed))
w = np.sort(np.array(walls[1:]))
print("SetNodes + SystemPlaceView over %d calls: p10 %.1f  median %.1f  p90 %.1f us"
      % (len(w), w[len(w) // 10], np.median(w), w[9 * len(w) // 10]))
st.close()
