import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
from nomad_amd import synth
from nomad_amd.stack import GenericStack
from tools import dropin
nodes, allocs = synth.cluster_c1(100, seed=42)
job = synth.mock_job(count=10)
orders = np.stack([synth.shuffle(len(nodes), 1 + e) for e in range(16)])
st = GenericStack()
st.SetState(nodes, allocs)
run = dropin.prepare(st, job)
run(orders, 10, n_evals=50)
for k in range(3):
    dropin.phase_seconds(reset=True)
    placed, ne, _, secs, _ = run(orders, 10, n_evals=2000)
    ph = dropin.phase_seconds(reset=True)
    print("us/eval %.2f" % (secs / ne * 1e6), {k: round(v / ne * 1e6, 2) for k, v in ph.items()}, flush=True)
print(st.SpeculationStats())
