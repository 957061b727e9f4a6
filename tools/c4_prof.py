"""k_system (SystemStack single-node Selects, grid-stride) against its
roofline: C4 clusters of growing size, the kernel's device time (HIP events on
the engine stream, median of 5) and the algorithmic bytes of SURVEY.md §8(d)
(73 B per node: 64 B NodeRec read + list entry + verdict byte, 9 B written:
FinalScore + outcome). Prints one JSON line per size. Used under rocprofv3
(tools/c4_pmc.sh) for the kernel stats and FETCH_SIZE / WRITE_SIZE."""
import json
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from nomad_amd import synth, synth_columnar  # noqa: E402
from nomad_amd.stack import SystemStack  # noqa: E402

sizes = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["100000", "400000", "1600000", "6400000"])]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
job = synth.mock_system_job()
for n in sizes:
    cs = synth_columnar.ColumnarState(n, seed=11, kind="c4", prefill=0.05)
    rows = np.random.Generator(np.random.PCG64(5)).permutation(n).astype(np.uint32)
    st = SystemStack()
    st.SetStateColumnar(cs)
    ks = []
    for i in range(reps):
        st.ResetPlan()
        st.SetJob(job)
        st.SetNodes(rows)
        st.SystemPlace(0)
        ks.append(st.last_kernel_ms())
    st.close()
    k = float(np.median(ks))
    print(json.dumps({"nodes": n, "k_system_ms": k, "bytes": n * 73, "GBps": n * 73 / (k * 1e-3) / 1e9,
                      "frac_of_8TBps": n * 73 / (k * 1e-3) / 8.0e12}), flush=True)
