#!/bin/bash
# Chain variant check: the chain-heavy GPU tests on the in-tree build, then the
# A/B timing against tools/ab/old (tools/ab_probe.sh). Outputs in gpurun_out/$1/.
set -eo pipefail
TAG=${1:-chk}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_chain_windows.py tests/test_dropin.py tests/test_engine_parity.py \
  tests/test_devices.py tests/test_golden.py tests/test_semantics.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash tools/ab_probe.sh "$TAG"
