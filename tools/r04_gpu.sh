#!/bin/bash
# Round-4 GPU check: pytest selection ($2, pytest -k expression or a file list
# in $3), then optional bench A/B of the chain shapes (set AB=1). Outputs in
# gpurun_out/<tag>/. Every GPU step has its own time limit; the script stops at
# the first failure.
set -eo pipefail
TAG=${1:-r04}
K=${2:-}
FILES=${3:-tests}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
ARGS=(-m gpu -x -v --timeout ${TEST_TIMEOUT:-120} --timeout-method thread --durations 15)
if [ -n "$K" ]; then ARGS+=(-k "$K"); fi
timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest $FILES "${ARGS[@]}" > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
grep -E "passed|failed" "$OUT/pytest.log" | tail -1
if [ -n "$AB" ]; then
  for SH in default unfused; do
    if [ "$SH" = default ]; then unset PE_CHAIN_FUSED; else export PE_CHAIN_FUSED=0; fi
    timeout -k 10 300 python -u bench.py --no-cpu --sweep-nodes 0 --sections ${SECTIONS:-c1} > "$OUT/b_$SH.json" 2> "$OUT/b_$SH.err" || { tail -20 "$OUT/b_$SH.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_$SH.json'));c=d['configs'];print('$SH', 'C2 %.4g' % d['value'], 'us/eval %.1f' % (d['ms_per_step']*1e3), ' '.join('%s %.4g' % (k, v.get('placements_per_s', v.get('nodes_per_s', 0))) for k, v in c.items()))"
  done
fi
