#!/bin/bash
# k_system evidence for DESIGN §3 / VERDICT r02 weak 5: kernel stats over a size
# sweep, then FETCH_SIZE and WRITE_SIZE (separate rocprofv3 passes) at 100k
# nodes. Outputs under gpurun_out/c4_pmc/.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/c4_pmc
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 240 python3 "$ROOT/tools/c4_prof.py" > "$OUT/sizes.jsonl" 2> "$OUT/sizes.err"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o stats -- \
  python3 "$ROOT/tools/c4_prof.py" 100000 5 > "$OUT/stats.jsonl" 2> "$OUT/stats.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- \
  python3 "$ROOT/tools/c4_prof.py" 100000 5 > "$OUT/f.jsonl" 2> "$OUT/f.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- \
  python3 "$ROOT/tools/c4_prof.py" 100000 5 > "$OUT/w.jsonl" 2> "$OUT/w.err"
cd "$ROOT"
F=$(find "$OUT/fetch" -name "*counter_collection.csv" -print -quit)
W=$(find "$OUT/write" -name "*counter_collection.csv" -print -quit)
python3 tools/pmc_traffic.py "$F" "$W" "k_system_rows" 100000 73 "$OUT/system_rows_traffic.json"
python3 tools/pmc_traffic.py "$F" "$W" "k_system_gather" 100000 21 "$OUT/system_gather_traffic.json" || true
cat "$OUT/sizes.jsonl"
find "$OUT/stats" -name "*kernel_stats.csv" -exec cp {} "$OUT/c4_kernel_stats.csv" \;
head -5 "$OUT/c4_kernel_stats.csv"
