"""Plan applier call-time probe (PE_PLAN_PROF=1 prints the host stages of
pe_planner_evaluate): the bench's 100k-node system-job plan."""
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from nomad_amd.plan import Planner  # noqa: E402
from nomad_amd.synth_plan import system_plan  # noqa: E402

nodes, allocs, plan = system_plan(100000, seed=42)
pl = Planner(0)
pl.set_state(nodes, allocs)
ep = pl.encode(plan)
for i in range(5):
    t0 = time.perf_counter()
    pl.evaluate(ep)
    print("call %.1f us, kernel %.1f us" % ((time.perf_counter() - t0) * 1e6, pl.kernel_ms() * 1e3), flush=True)
pl.close()
