"""C4 drop-in probe (GPU box): the SystemScheduler caller loop of
bench.py's c4_drop_in on 100k nodes, the loop's phases per evaluation, and
with PE_API_PROF=1 the engine's host steps (printed when the stack closes)."""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from nomad_amd import synth, synth_columnar  # noqa: E402
from nomad_amd.stack import SystemStack  # noqa: E402
from tools import dropin  # noqa: E402

n = 100000
cs = synth_columnar.ColumnarState(n, seed=11, kind="c4", prefill=0.05)
job = synth.mock_system_job()
rows = np.random.Generator(np.random.PCG64(5)).permutation(n).astype(np.uint32)
st = SystemStack()
st.SetStateColumnar(cs)
evals = int(sys.argv[1]) if len(sys.argv) > 1 else 6
for i in range(evals):
    dropin.system_phases(reset=True)
    st.ResetPlan()
    st.SetJob(job)
    _, _, placed, secs = dropin.system_loop(st, 0, rows)
    ph = dropin.system_phases(reset=True)
    print("eval %d: %.3f ms, placed %d, %s" % (i, secs * 1e3, placed, {k: round(v * 1e3, 3) for k, v in ph.items()}),
          flush=True)
st.close()
