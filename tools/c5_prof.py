"""C5 count loop on one GPU (profiling driver): 2 x nvidia/gpu count=1000 on
50k nodes with service preemption, 99 % of the GPU nodes busy.
Usage: c5_prof.py [runs] (default 2); PE_ENGINE_LIB picks the library (A/B)."""
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from nomad_amd import synth  # noqa: E402
from nomad_amd.stack import GenericStack  # noqa: E402
from nomad_amd.structs import SchedulerConfig  # noqa: E402

nodes, allocs = synth.cluster_c5(50000, seed=5, busy=0.99)
job = synth.job_c5(1000)
perm = synth.shuffle(len(nodes), 77)
st = GenericStack(config=SchedulerConfig(preempt_service=True))
st.SetState(nodes, allocs)
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 2
ms = []
for i in range(runs):
    st.ResetPlan()
    st.SetJob(job)
    st.SetNodes(perm)
    t0 = time.perf_counter()
    res = st.Place(0, 1000)
    ms.append((time.perf_counter() - t0) * 1e3)
    print("run", i, "ms", ms[-1], "preempting", sum(1 for r in res if r.preempted))
warm = sorted(ms[1:]) or ms
print("min %.2f median %.2f ms over %d warm runs" % (warm[0], warm[len(warm) // 2], len(warm)))
