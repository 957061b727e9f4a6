#!/bin/bash
# Plan applier profile on the GPU box: the bench's plan_apply section alone,
# its rocprofv3 kernel trace + stats, and FETCH_SIZE / WRITE_SIZE passes
# (separate runs) summarised per k_plan_eval launch. Outputs in gpurun_out/<tag>/.
set -eo pipefail
TAG=${1:-planprof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --evals 1 --sweep-nodes 0 --sections plan_apply \
  > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(json.dumps(d['configs']['plan_apply'],indent=1))"
cd /tmp
export TMPDIR=/tmp
ARGS="--no-cpu --steps 1 --warmup 0 --evals 1 --sweep-nodes 0 --sections plan_apply"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o plan -- \
  python3 "$ROOT/bench.py" $ARGS > "$OUT/trace.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o fetch -- \
  python3 "$ROOT/bench.py" $ARGS > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o write -- \
  python3 "$ROOT/bench.py" $ARGS > "$OUT/pmc_write.log" 2>&1
cd "$ROOT"
find "$OUT" -name "*kernel_stats.csv" -exec grep -h "plan_eval\|Name" {} \;
BYTES=$(python3 -c "import json;print(json.load(open('$OUT/bench.json'))['configs']['plan_apply']['roofline']['bytes_per_launch_rank0'])")
F=$(find "$OUT/pmc_fetch" -name "*counter_collection.csv" -print -quit)
W=$(find "$OUT/pmc_write" -name "*counter_collection.csv" -print -quit)
python3 tools/pmc_traffic.py "$F" "$W" "k_plan_eval" "$BYTES" 1 "$OUT/plan_traffic.json"
cat "$OUT/plan_traffic.json"
