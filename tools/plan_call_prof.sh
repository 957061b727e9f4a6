#!/bin/bash
# Where the plan applier call's time goes (PE_PLAN_PROF): strings, flatten,
# plan-node records, uploads, kernel + reasons, for the bench's 100k-node
# system plan, over worker / chunk / spin settings ($PLAN_AB: space-separated
# env assignments joined by commas, "default" for none). Outputs in
# gpurun_out/<tag>/.
set -eo pipefail
TAG=${1:-planprof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
echo "nproc $(nproc) cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo n/a) affinity $(python3 -c 'import os;print(len(os.sched_getaffinity(0)))')"
for V in ${PLAN_AB:-default}; do
  if [ "$V" = default ]; then E=""; else E="${V//,/ }"; fi
  env $E PE_PLAN_PROF=1 timeout -k 10 300 python -u bench.py --no-cpu --steps 2 --warmup 1 --sweep-nodes 0 --sections plan_apply \
    > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
  echo "== $V"
  grep "planner evaluate" "$OUT/bench.err" | tail -2
  python3 -c "import json;d=json.load(open('$OUT/bench.json'));p=d['configs']['plan_apply'];print('call_ms %.3f kernel_ms %.4f' % (p['call_ms'], p['kernel_ms']))"
done
