"""AllocMetric-on drop-in probe (GPU box): the headline caller loop (C2, 10k
nodes, count 1000) with pe_set_metrics on and the maps copied out by the
caller; per evaluation wall time, and with PE_METRICS_PROF=1 the speculative
run's metric phases (host walk, k_trace, maps + text)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from nomad_amd import synth  # noqa: E402
from nomad_amd.stack import GenericStack  # noqa: E402
from tools import dropin  # noqa: E402

n, count = 10000, 1000
kind = sys.argv[1] if len(sys.argv) > 1 else "c2"
preempt = kind == "c5"
cfg = None
if kind == "c5":   # evicting runs (the replayed maps)
    from nomad_amd.structs import SchedulerConfig
    n = 50000
    nodes, allocs = synth.cluster_c5(n, seed=5, busy=0.99)
    job = synth.job_c5(count)
    cfg = SchedulerConfig(preempt_service=True)
elif kind == "c3":   # spread + affinity full passes (the batched spread trace)
    nodes, allocs = synth.cluster_c3(n, seed=7)
    job = synth.job_c3(count)
else:
    nodes, allocs = synth.cluster_c2(n, seed=42)
    job = synth.job_c2(count)
orders = np.stack([synth.shuffle(n, 1000 + e) for e in range(8)])
st = GenericStack(config=cfg) if cfg else GenericStack()
st.SetState(nodes, allocs)
st.EnableMetrics(True)
dropin.use_metrics(True)
caller = dropin.prepare(st, job)
caller(orders, count, preempt=preempt, n_evals=1)
for i in range(2 if preempt else 4):
    dropin.phase_seconds(reset=True)
    t0 = time.perf_counter()
    placed, ne, _, _, _ = caller(orders, count, preempt=preempt, n_evals=int(os.environ.get("PROBE_EVALS", "2")))
    dt = time.perf_counter() - t0
    ph = dropin.phase_seconds(reset=True)
    print("%.3f ms per evaluation" % (dt / ne * 1e3), {k: round(v / ne * 1e3, 3) for k, v in ph.items()}, flush=True)
