#!/bin/bash
# A/B timing of two trees on one box: a built copy of an earlier commit under
# tools/ab/old/ (A, not tracked) against the in-tree build (B), interleaved,
# C2 and C1 drop-in loops and the k_chain step clocks. Outputs in gpurun_out/$1/.
set -eo pipefail
TAG=${1:-ab}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for round in 1 2; do
  for v in a b; do
    if [ $v = a ]; then P=tools/ab/old/tools/dropin_probe.py; else P=tools/dropin_probe.py; fi
    timeout -k 10 120 python -u $P 10000 1000 300 > "$OUT/c2_${v}${round}.txt" 2>&1 || { tail -20 "$OUT/c2_${v}${round}.txt"; exit 1; }
    timeout -k 10 120 python -u $P 100 10 3000 > "$OUT/c1_${v}${round}.txt" 2>&1 || { tail -20 "$OUT/c1_${v}${round}.txt"; exit 1; }
    echo "== $v round $round"; head -1 "$OUT/c2_${v}${round}.txt"; grep "k_chain phase" "$OUT/c2_${v}${round}.txt" | tail -2; head -1 "$OUT/c1_${v}${round}.txt"; grep "k_chain phase" "$OUT/c1_${v}${round}.txt" | tail -1
  done
done
