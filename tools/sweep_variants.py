"""Scoring-sweep variants on the 2^24-node C3-like columnar cluster: median
kernel time per full-scan Select for PE_SWEEP_VARIANT x PE_SWEEP_BPC, and the
same winner across all of them."""
import itertools
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from nomad_amd import synth, synth_columnar  # noqa: E402
from nomad_amd.stack import GenericStack  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
variants = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "2", "3", "4"]
bpcs = sys.argv[3].split(",") if len(sys.argv) > 3 else ["0"]
t0 = time.perf_counter()
cs = synth_columnar.ColumnarState(n, seed=7, kind="c3")
st = GenericStack()
st.SetStateColumnar(cs)
st.SetJob(synth.job_c3(1000))
st.SetNodes(np.random.Generator(np.random.PCG64(3)).permutation(n).astype(np.uint32))
print("setup %.1f s" % (time.perf_counter() - t0), flush=True)
rows = set()
for v, b in itertools.product(variants, bpcs):
    os.environ["PE_SWEEP_VARIANT"] = v
    if v == "noaux":
        os.environ["PE_SWEEP_AUX"] = "0"
        os.environ["PE_SWEEP_VARIANT"] = "0"
    else:
        os.environ.pop("PE_SWEEP_AUX", None)
    if b == "0":
        os.environ.pop("PE_SWEEP_BPC", None)
    else:
        os.environ["PE_SWEEP_BPC"] = b
    ms = []
    for i in range(6):
        r = st.SelectRaw(0)
        if i:
            ms.append(st.last_kernel_ms())
    if v not in ("5", "6", "7", "8"):
        rows.add((r.row, r.final_score))
    k = float(np.median(ms))
    bpn = st.last_sweep_bytes()
    print("variant %s bpc %s: %.4f ms  %.2f TB/s (%d B/node)  row %d" % (v, b, k, n * bpn / k / 1e9, bpn, r.row),
          flush=True)
assert len(rows) == 1, rows
print("same winner everywhere", rows)
