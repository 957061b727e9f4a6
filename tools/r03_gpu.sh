#!/bin/bash
# Round-3 GPU pass: the whole -m gpu suite, the default bench line, then the
# C4 k_system evidence (size sweep, kernel stats, FETCH/WRITE passes).
# Outputs in gpurun_out/$1/ (default r03).
set -eo pipefail
TAG=${1:-r03}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
PE_PLACE_PROF=1 timeout -k 10 180 python -u tools/c5_prof.py > "$OUT/c5_prof.txt" 2>&1 || { tail -30 "$OUT/c5_prof.txt"; exit 1; }
cat "$OUT/c5_prof.txt"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
head -c 3000 "$OUT/bench.json"; echo
bash tools/c4_pmc.sh
