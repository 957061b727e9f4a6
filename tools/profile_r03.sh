#!/bin/bash
# Round-3 profile on the GPU box. Order: the PMC passes first (FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 runs) over the headline loop and the
# 2^24-node scoring sweep, summarised per launch
# (tools/pmc_traffic.py) and copied to profiles/r03/ where bench.py reads them;
# then the default bench line, the rocprofv3 kernel stats + device timeline of
# the headline loop, and the kernel stats of the C5 and C3 loops. Every GPU
# step has its own time limit; the script stops at the first failure. Outputs
# in gpurun_out/<tag>/ (copied into profiles/r03/ by hand afterwards).
set -eo pipefail
TAG=${1:-r03p}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT" "$ROOT/profiles/r03"
cd "$ROOT"
bash tools/headline_pmc.sh
cp gpurun_out/headline_pmc/headline_traffic.json "$OUT/" && cp "$OUT/headline_traffic.json" profiles/r03/
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o fetch -- \
  python3 "$ROOT/tools/sweep_variants.py" 16777216 0 0 > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o write -- \
  python3 "$ROOT/tools/sweep_variants.py" 16777216 0 0 > "$OUT/pmc_write.log" 2>&1
cd "$ROOT"
F=$(find "$OUT/pmc_fetch" -name "*counter_collection.csv" -print -quit)
W=$(find "$OUT/pmc_write" -name "*counter_collection.csv" -print -quit)
python3 tools/pmc_traffic.py "$F" "$W" "k_sweep<" 16777216 76 "$OUT/sweep_traffic.json"
cp "$OUT/sweep_traffic.json" profiles/r03/
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value', d['value'], 'cpu', d['cpu_baseline']['value'], 'traffic', d['roofline']['traffic'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 10 --warmup 2 --sweep-nodes 0 --sections "" > "$OUT/trace.log" 2>&1
T=$(find "$OUT/trace" -name "*kernel_trace.csv" -print -quit)
python3 "$ROOT/tools/timeline.py" "$T" k_emit_writeback 3 > "$OUT/headline_timeline.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5" -o c5 -- \
  python3 "$ROOT/tools/c5_prof.py" > "$OUT/c5.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3" -o c3 -- \
  python3 "$ROOT/tools/c3_loop_probe.py" 10000 1000 > "$OUT/c3.log" 2>&1
cat "$OUT/c5.log" "$OUT/c3.log"
find "$OUT" -name "*kernel_stats.csv" | sort
