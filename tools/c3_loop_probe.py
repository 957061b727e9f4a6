"""C3 count-loop probe: fused pe_place (one workgroup per eval) against a
host-driven Select+Commit loop whose Selects use the multi-CU sweep
(PE_SWEEP_MIN set by the caller). Prints ms per placement and checks rows agree."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nomad_amd import synth  # noqa: E402
from nomad_amd.stack import GenericStack  # noqa: E402

n, count = int(sys.argv[1]), int(sys.argv[2])
nodes, allocs = synth.cluster_c3(n, seed=7)
job = synth.job_c3(count)
perm = list(synth.shuffle(n, 3))
st = GenericStack()
st.SetState(nodes, allocs)
st.SetJob(job)
st.SetNodes(perm)
st.Place(0, count)
st.ResetPlan(); st.SetJob(job); st.SetNodes(perm)
t0 = time.perf_counter()
fused = st.Place(0, count)
t_f = time.perf_counter() - t0
st.ResetPlan(); st.SetJob(job); st.SetNodes(perm)
rows = []
t0 = time.perf_counter()
for k in range(count):
    r = st.Select(0)
    if r is None:
        break
    st.Commit(0, r.row)
    rows.append(r.row)
t_s = time.perf_counter() - t0
print("n=%d count=%d fused %.1f us/placement, select+commit loop %.1f us/placement, same rows %s"
      % (n, count, t_f / count * 1e6, t_s / count * 1e6, rows == [x.row for x in fused][:len(rows)]))
