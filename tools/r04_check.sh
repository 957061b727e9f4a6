#!/bin/bash
# Round-4 GPU check: new tests first (-k $2 or the files in $3), then the whole
# -m gpu suite, then a short bench of the sections in $SECTIONS. Every GPU step
# has its own time limit; the script stops at the first failure. Outputs in
# gpurun_out/<tag>/.
set -eo pipefail
TAG=${1:-r04c}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
ARGS=(-m gpu -x -v --timeout 300 --timeout-method thread --durations 15)
if [ -n "$FIRST" ]; then
  timeout -k 10 600 python -u -m pytest $FIRST "${ARGS[@]}" > "$OUT/first.log" 2>&1 || { tail -80 "$OUT/first.log"; exit 1; }
  grep -E "passed|failed" "$OUT/first.log" | tail -1
fi
if [ -z "$NO_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations 20 \
    > "$OUT/gpu_pytest.log" 2>&1 || { tail -80 "$OUT/gpu_pytest.log"; exit 1; }
  tail -1 "$OUT/gpu_pytest.log"
fi
if [ -n "$SECTIONS" ]; then
  timeout -k 10 400 python -u bench.py --no-cpu --sweep-nodes 0 --sections "$SECTIONS" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('C2 %.4g' % d['value'], 'us/eval %.1f' % (d['ms_per_step']*1e3)); print(' '.join('%s %.4g' % (k, v.get('placements_per_s', v.get('nodes_per_s', 0))) for k, v in d['configs'].items() if isinstance(v, dict)))"
fi
if [ -n "$AB_LIBS" ]; then   # A/B of engine builds: the C5 loop (tools/c5_prof.py) with each
  for LIB in $AB_LIBS; do
    if [ "$LIB" = default ]; then unset PE_ENGINE_LIB; else export PE_ENGINE_LIB=$ROOT/$LIB; fi
    echo "== $LIB"
    PE_PLACE_PROF=1 timeout -k 10 300 python -u tools/c5_prof.py > "$OUT/ab_$(basename $LIB).txt" 2>&1 || { tail -20 "$OUT/ab_$(basename $LIB).txt"; exit 1; }
    grep -E "^run|k_ploop:" "$OUT/ab_$(basename $LIB).txt" | tail -4
  done
  unset PE_ENGINE_LIB
fi
if [ -n "$CHAIN_PROF" ]; then   # k_chain per-step clock profile of the C2 loop
  timeout -k 10 200 python -u tools/chain_prof.py > "$OUT/chain_prof.txt" 2>&1 || { tail -20 "$OUT/chain_prof.txt"; exit 1; }
  tail -12 "$OUT/chain_prof.txt"
fi
if [ -n "$C1_TRACE" ]; then   # device timeline of the C1 evaluation loop
  cd /tmp
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c1trace" -o c1 -- \
    python3 "$ROOT/bench.py" --no-cpu --steps 3 --warmup 1 --sweep-nodes 0 --sections c1 > "$OUT/c1trace.log" 2>&1
  cd "$ROOT"
  T=$(find "$OUT/c1trace" -name "*kernel_trace.csv" -print -quit)
  python3 tools/timeline.py "$T" k_chain 4 > "$OUT/c1_timeline.txt" || true
  tail -24 "$OUT/c1_timeline.txt"
fi
if [ -n "$AB_ENV" ]; then   # headline bench A/B: default vs the environment settings in $AB_ENV
  for V in default "$AB_ENV"; do
    if [ "$V" = default ]; then E=""; else E="$V"; fi
    env $E timeout -k 10 300 python -u bench.py --no-cpu --sweep-nodes 0 --sections "" > "$OUT/ab_env.json" 2> "$OUT/ab_env.err" || { tail -20 "$OUT/ab_env.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/ab_env.json'));print('$V', 'C2 %.4g' % d['value'], 'us/eval %.1f' % (d['ms_per_step']*1e3), d['drop_in']['us_per_eval_by_phase'])"
  done
fi
