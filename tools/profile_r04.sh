#!/bin/bash
# Round-4 GPU pass: the -m gpu suite, the FETCH_SIZE calibration, the default
# bench line, then rocprofv3 kernel stats of the headline loop (with its device
# timeline), of the 2^24-node scoring sweep and of the C5 loop, and the PMC
# traffic passes of the headline evaluation (tools/headline_pmc_r04.sh) and of
# the sweep (FETCH_SIZE x 2, the calibrated 16-B streaming factor). Every GPU step has its own time limit; the
# script stops at the first failure. Outputs in gpurun_out/<tag>/ (copied into
# profiles/r04/ by hand afterwards). SKIP_TESTS=1 skips the suite.
set -eo pipefail
TAG=${1:-r04p}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations 20 \
    > "$OUT/gpu_pytest.log" 2>&1 || { tail -60 "$OUT/gpu_pytest.log"; exit 1; }
  tail -1 "$OUT/gpu_pytest.log"
fi
cd /tmp
export TMPDIR=/tmp
for R in 10000 1048576; do
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_f$R" -o f -- \
    "$ROOT/tools/fetch_calib" $R > "$OUT/calib_$R.txt" 2> "$OUT/calib_f$R.err"
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib_w$R" -o w -- \
    "$ROOT/tools/fetch_calib" $R > /dev/null 2> "$OUT/calib_w$R.err"
  python3 "$ROOT/tools/fetch_calib.py" $(find "$OUT/calib_f$R" -name "*counter_collection.csv" -print -quit) \
    $(find "$OUT/calib_w$R" -name "*counter_collection.csv" -print -quit) "$OUT/calib_$R.txt" "$OUT/fetch_calib_$R.json" > /dev/null
done
cd "$ROOT"
timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print('value %.4g' % d['value'], 'us/eval %.1f' % (d['ms_per_step']*1e3), 'cpu', d['cpu_baseline']['value'], 'frac', r['frac'], 'traffic', r['traffic']); print(' '.join('%s %.4g' % (k, v.get('placements_per_s', v.get('nodes_per_s', 0))) for k, v in d['configs'].items() if isinstance(v, dict)))"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 10 --warmup 2 --sweep-nodes 0 --sections "" > "$OUT/trace.log" 2>&1
T=$(find "$OUT/trace" -name "*kernel_trace.csv" -print -quit)
python3 "$ROOT/tools/timeline.py" "$T" k_emit_writeback 3 > "$OUT/headline_timeline.txt" || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/sweep" -o sweep -- \
  python3 "$ROOT/tools/sweep_variants.py" 16777216 0 0 > "$OUT/sweep.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5" -o c5 -- \
  python3 "$ROOT/tools/c5_prof.py" > "$OUT/c5.log" 2>&1
cat "$OUT/sweep.log" "$OUT/c5.log" | tail -20
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/sweep_f" -o f -- \
  python3 "$ROOT/tools/sweep_variants.py" 16777216 0 0 > /dev/null 2> "$OUT/sweep_f.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/sweep_w" -o w -- \
  python3 "$ROOT/tools/sweep_variants.py" 16777216 0 0 > /dev/null 2> "$OUT/sweep_w.err"
cd "$ROOT"
python3 tools/pmc_traffic.py $(find "$OUT/sweep_f" -name "*counter_collection.csv" -print -quit) \
  $(find "$OUT/sweep_w" -name "*counter_collection.csv" -print -quit) "k_sweep<" 16777216 76 "$OUT/sweep_traffic.json" 2.0 \
  | grep -E "traffic_over|bytes_per_launch"
bash tools/headline_pmc_r04.sh | grep -E "traffic_over|k_base_bytes|k_chain_bytes"
cp gpurun_out/headline_pmc/headline_traffic.json "$OUT/headline_traffic.json"
find "$OUT" -name "*kernel_stats.csv" | sort
