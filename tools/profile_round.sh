#!/bin/bash
# Round profile on the GPU box: default bench line (with CPU baseline), the
# rocprofv3 kernel trace + stats of the same bench, and the two PMC passes
# (FETCH_SIZE, WRITE_SIZE) over the 2^24-node scoring sweep, summarised into
# per-launch HBM traffic. Every GPU step has its own time limit; the script
# stops at the first failure. Outputs land in gpurun_out/<tag>/.
set -eo pipefail
TAG=${1:-prof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 10 --warmup 2 --sections "" > "$OUT/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o fetch -- \
  python3 "$ROOT/tools/sweep_variants.py" 16777216 0 0 > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o write -- \
  python3 "$ROOT/tools/sweep_variants.py" 16777216 0 0 > "$OUT/pmc_write.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/chain_fetch" -o fetch -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 2 --warmup 0 --sweep-nodes 0 --sections "" > "$OUT/chain_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/chain_write" -o write -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 2 --warmup 0 --sweep-nodes 0 --sections "" > "$OUT/chain_write.log" 2>&1
cd "$ROOT"
EV=$(python3 -c "import json;print(int(json.load(open('$OUT/bench.json'))['roofline']['node_evals_per_launch']))")
CF=$(find "$OUT/chain_fetch" -name "*counter_collection.csv" -print -quit)
CW=$(find "$OUT/chain_write" -name "*counter_collection.csv" -print -quit)
python3 tools/pmc_traffic.py "$CF" "$CW" "k_chain" "$EV" 60 "$OUT/chain_traffic.json"
F=$(find "$OUT/pmc_fetch" -name "*counter_collection.csv" -print -quit)
W=$(find "$OUT/pmc_write" -name "*counter_collection.csv" -print -quit)
python3 tools/pmc_traffic.py "$F" "$W" "k_sweep<" 16777216 76 "$OUT/sweep_traffic.json"
find "$OUT" -name "*.csv" | sort
