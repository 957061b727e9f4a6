#!/bin/bash
# One GPU-box session: parity tests, bench eval-count sweep, rocprofv3 kernel
# trace (CSV), SQ counters on the count-loop kernel and HBM counters on the
# 2^24-node scoring sweep. Every GPU step has its own time limit; the script
# stops at the first failure. Outputs land in gpurun_out/<tag>/.
set -eo pipefail
TAG=${1:-run}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1
tail -2 "$OUT/pytest_gpu.log"
for E in 2048 4096 8192; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --evals $E --no-cpu --sweep-nodes 0 > "$OUT/b$E.json" 2> "$OUT/b$E.err"
  python -c "import json;d=json.load(open('$OUT/b$E.json'));print($E, round(d['value']/1e6,1), d['step_phases_ms'])"
done
[ "${2:-}" = quick ] && exit 0
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 5 --evals 4096 > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  --output-format csv -d "$OUT/pmc_sq" -o sq -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 2 --warmup 1 --evals 4096 --sweep-nodes 0 > "$OUT/pmc_sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o fetch -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 1 --warmup 0 --evals 64 > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o write -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 1 --warmup 0 --evals 64 > "$OUT/pmc_write.log" 2>&1
find "$OUT" -name "*.csv" | sort
