#!/bin/bash
# Iteration check: the whole -m gpu suite, then the latency probes
# (tools/r03_probe.sh). Outputs in gpurun_out/$1/.
set -eo pipefail
TAG=${1:-iter}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
bash tools/r03_probe.sh "$TAG"
