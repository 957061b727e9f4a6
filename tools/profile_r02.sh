#!/bin/bash
# Round-2 profile on the GPU box: the default bench line (CPU baselines
# included), rocprofv3 kernel stats of the bench's headline loop, of the C5
# loop (k_ploop) and of the C3 count loop, the device timeline of three
# headline evaluations (tools/timeline.py), and the PMC traffic passes
# (FETCH_SIZE, WRITE_SIZE in separate runs) of the 2^24-node scoring sweep.
# Every GPU step has its own time limit; the script stops at the first
# failure. Outputs land in gpurun_out/<tag>/.
set -eo pipefail
TAG=${1:-r02}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value', d['value'], 'cpu', d['cpu_baseline']['value'])"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 10 --warmup 2 --sweep-nodes 0 --sections "" > "$OUT/trace.log" 2>&1
T=$(find "$OUT/trace" -name "*kernel_trace.csv" -print -quit)
python3 "$ROOT/tools/timeline.py" "$T" k_emit_writeback 3 > "$OUT/headline_timeline.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5" -o c5 -- \
  python3 "$ROOT/tools/c5_prof.py" > "$OUT/c5.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3" -o c3 -- \
  python3 "$ROOT/tools/c3_loop_probe.py" 10000 1000 > "$OUT/c3.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o fetch -- \
  python3 "$ROOT/tools/sweep_variants.py" 16777216 0 0 > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o write -- \
  python3 "$ROOT/tools/sweep_variants.py" 16777216 0 0 > "$OUT/pmc_write.log" 2>&1
cd "$ROOT"
F=$(find "$OUT/pmc_fetch" -name "*counter_collection.csv" -print -quit)
W=$(find "$OUT/pmc_write" -name "*counter_collection.csv" -print -quit)
python3 tools/pmc_traffic.py "$F" "$W" "k_sweep<" 16777216 76 "$OUT/sweep_traffic.json"
cat "$OUT/c5.log" "$OUT/c3.log"
find "$OUT" -name "*kernel_stats.csv" | sort
