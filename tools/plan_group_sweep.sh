#!/bin/bash
# k_plan_eval group-size sweep on the GPU box: parity tests and the bench's
# plan_apply section per PE_PLAN_GROUP. Outputs in gpurun_out/<tag>/.
set -eo pipefail
TAG=${1:-plangroups}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for G in 4 8 16 64; do
  PE_PLAN_GROUP=$G timeout -k 10 200 python -u -m pytest tests/test_plan_apply.py -x -q -m gpu --timeout 120 \
    --timeout-method thread > "$OUT/pytest_$G.log" 2>&1
  tail -1 "$OUT/pytest_$G.log"
  PE_PLAN_GROUP=$G timeout -k 10 200 python -u bench.py --no-cpu --steps 1 --warmup 0 --evals 1 --sweep-nodes 0 \
    --sections plan_apply > "$OUT/bench_$G.json" 2> "$OUT/bench_$G.err"
  python3 -c "import json;d=json.load(open('$OUT/bench_$G.json'))['configs']['plan_apply'];print($G, 'kernel_ms', d['kernel_ms'], 'nodes/s %.3g' % d['plan_nodes_per_s'])"
done
