"""Plan applier timing probe: evaluate and commit (pe_planner_commit) of a
system-job plan on an n-node snapshot; C calls timed, Python flattening done first."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from nomad_amd import abi  # noqa: E402
from nomad_amd.plan import Planner, _p  # noqa: E402
from nomad_amd.synth_plan import system_plan  # noqa: E402

n = int(sys.argv[1])
sub = int(sys.argv[2]) if len(sys.argv) > 2 else 0   # plan only the first `sub` nodes (0: all)
nodes, allocs, plan = system_plan(n, seed=42)
if sub:
    keep_ids = [nd.id for nd in nodes[:sub]]
    plan.node_allocation = {k: plan.node_allocation[k] for k in keep_ids}
pl = Planner()
pl.set_state(nodes, allocs)
ep = pl.encode(plan)
codes = pl.evaluate(ep)
keep = np.asarray([c == abi.PE_PLAN_FIT for c in codes], dtype=np.uint8)
t0 = time.perf_counter()
codes = pl.evaluate(ep)
t_eval = time.perf_counter() - t0
t0 = time.perf_counter()
rc = pl.lib.pe_planner_commit(pl.h, C.byref(ep.strtab), C.byref(ep.c), _p(keep, abi.u8p))
t_commit = time.perf_counter() - t0
assert rc == 0
print("plan nodes=%d " % len(ep.node_ids) + "n=%d evaluate %.2f ms (kernel %.3f ms), commit %.2f ms, snapshot allocs %d"
      % (n, t_eval * 1e3, pl.kernel_ms(), t_commit * 1e3, pl.lib.pe_planner_snapshot_allocs(pl.h)))
