"""Per-step clock profile of k_chain on the C2 workload (PE_CHAIN_PROF=1)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PE_CHAIN_PROF"] = "1"
from nomad_amd import synth  # noqa: E402
from nomad_amd.stack import GenericStack  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
count = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
nodes, allocs = synth.cluster_c2(n, seed=42)
job = synth.job_c2(count)
st = GenericStack()
st.SetState(nodes, allocs)
for i in range(3):
    st.ResetPlan()
    st.SetJob(job)
    st.SetNodes(synth.shuffle(n, 1000 + i))
    t = time.perf_counter()
    st.PlaceArrays(0, count)
    print("wall %.3f ms kernel %.3f ms" % ((time.perf_counter() - t) * 1e3, st.last_kernel_ms()), flush=True)
