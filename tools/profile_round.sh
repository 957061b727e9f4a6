#!/bin/bash
# Round profile on the GPU box, in two calls (the default bench line runs for
# minutes with its CPU baselines):
#   profile_round.sh <tag> bench   the default bench line (with CPU baselines)
#   profile_round.sh <tag> prof    rocprofv3 kernel trace + stats of the
#                                  headline bench and of the C5 count loop,
#                                  the headline's HBM traffic (headline_pmc.sh)
#                                  and the 2^24-node sweep's (FETCH_SIZE and
#                                  WRITE_SIZE in separate passes)
# Every GPU step has its own time limit; the script stops at the first
# failure. Outputs land in gpurun_out/<tag>/.
set -eo pipefail
TAG=${1:-prof}
MODE=${2:-prof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ "$MODE" = bench ]; then
  timeout -k 10 900 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
  cat "$OUT/bench.json"
  exit 0
fi
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 10 --warmup 2 --sections "" > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5trace" -o c5 -- \
  python3 "$ROOT/tools/c5_prof.py" 4 > "$OUT/c5trace.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3trace" -o c3 -- \
  python3 "$ROOT/tools/c3_full_prof.py" > "$OUT/c3trace.log" 2>&1
cd "$ROOT"
bash tools/headline_pmc.sh > "$OUT/headline_pmc.log" 2>&1
cp gpurun_out/headline_pmc/headline_traffic.json "$OUT/headline_traffic.json"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o fetch -- \
  python3 "$ROOT/tools/sweep_variants.py" 16777216 0 0 > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o write -- \
  python3 "$ROOT/tools/sweep_variants.py" 16777216 0 0 > "$OUT/pmc_write.log" 2>&1
cd "$ROOT"
F=$(find "$OUT/pmc_fetch" -name "*counter_collection.csv" -print -quit)
W=$(find "$OUT/pmc_write" -name "*counter_collection.csv" -print -quit)
python3 tools/pmc_traffic.py "$F" "$W" "k_sweep<" 16777216 76 "$OUT/sweep_traffic.json"
find "$OUT" -name "*stats.csv" | sort
