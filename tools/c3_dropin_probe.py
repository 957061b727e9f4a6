"""C3 drop-in probe (GPU box): the bench's C3 evaluation through the C caller
loop with the served-Select view; per-evaluation wall and (PE_API_PROF=1) the
engine's host steps, printed when the stack closes."""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from nomad_amd import synth  # noqa: E402
from nomad_amd.stack import GenericStack  # noqa: E402
from tools import dropin  # noqa: E402

nodes, allocs = synth.cluster_c3(10000, seed=7)
job = synth.job_c3(1000)
perm = np.asarray(synth.shuffle(len(nodes), 17), dtype=np.uint32)[None, :]
st = GenericStack()
st.SetState(nodes, allocs)
run = dropin.prepare(st, job)
for i in range(4):
    dropin.phase_seconds(reset=True)
    placed, _, _, dt, _ = run(perm, 1000)
    ph = dropin.phase_seconds(reset=True)
    print("%.3f ms per evaluation" % (dt * 1e3), {k: round(v * 1e3, 3) for k, v in ph.items()},
          st.SpeculationStats(), flush=True)
st.close()
