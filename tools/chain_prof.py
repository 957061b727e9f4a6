"""Per-step clock profile of k_chain on the C2 workload (PE_CHAIN_PROF=1).
Usage: chain_prof.py [n] [count] [runs]; NOPROF=1 times the kernels without
the step profile (PE_ENGINE_LIB picks the library for A/B)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if not os.environ.get("NOPROF"):
    os.environ["PE_CHAIN_PROF"] = "1"
from nomad_amd import synth  # noqa: E402
from nomad_amd.stack import GenericStack  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
count = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
nodes, allocs = synth.cluster_c2(n, seed=42)
job = synth.job_c2(count)
st = GenericStack()
st.SetState(nodes, allocs)
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 3
ks = []
for i in range(runs):
    st.ResetPlan()
    st.SetJob(job)
    st.SetNodes(synth.shuffle(n, 1000 + i))
    t = time.perf_counter()
    st.PlaceArrays(0, count)
    ks.append(st.last_kernel_ms())
    print("wall %.3f ms kernel %.3f ms" % ((time.perf_counter() - t) * 1e3, ks[-1]), flush=True)
warm = sorted(ks[1:]) or ks
print("kernel min %.4f median %.4f ms over %d warm runs" % (warm[0], warm[len(warm) // 2], len(warm)))
