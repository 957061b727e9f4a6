"""Single-evaluation latency breakdown of the C2 count loop (host call phases)."""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from nomad_amd import synth  # noqa: E402
from nomad_amd.stack import GenericStack  # noqa: E402

nodes, allocs = synth.cluster_c2(10000, seed=42)
job = synth.job_c2(1000)
perm = synth.shuffle(len(nodes), 1000)
st = GenericStack()
st.SetState(nodes, allocs)
ph = {"reset": [], "setjob": [], "setnodes": [], "place": [], "kernel": []}
for i in range(12):
    t0 = time.perf_counter(); st.ResetPlan(); t1 = time.perf_counter()
    st.SetJob(job); t2 = time.perf_counter()
    st.SetNodes(perm); t3 = time.perf_counter()
    st.PlaceArrays(0, 1000); t4 = time.perf_counter()
    if i >= 2:
        for k, v in zip(ph, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, st.last_kernel_ms() / 1e3)):
            ph[k].append(v * 1e3)
print({k: round(float(np.median(v)), 4) for k, v in ph.items()})
