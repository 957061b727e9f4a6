#!/bin/bash
# Short GPU-box check: parity tests matching $2 (pytest -k, default all gpu tests)
# and bench lines at a few concurrent-eval counts. Outputs in gpurun_out/$1/.
set -eo pipefail
TAG=${1:-quick}
K=${2:-}
EVALS=${3:-"1 4096"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
else
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
fi
tail -1 "$OUT/pytest.log"
for E in $EVALS; do
  timeout -k 10 200 python -u bench.py --no-cpu --sweep-nodes 0 --evals $E > "$OUT/b$E.json" 2> "$OUT/b$E.err" || { tail -20 "$OUT/b$E.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b$E.json'));print($E, 'value %.4g' % d['value'], 'kernel_ms', d['step_phases_ms']['kernel'], 'single', '%.4g' % d['single_eval']['placements_per_s'], d['single_eval']['kernel_ms'])"
done
