#!/bin/bash
# HBM traffic of the batched C2 launch (bench.py section c2_batch: 4096
# evaluations per pe_place_batch, one k_base pass + the batched k_chain):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes, combined per launch by
# tools/pmc_traffic.py. Writes gpurun_out/batch_pmc/c2_batch_traffic.json.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/batch_pmc
mkdir -p "$OUT"
cd "$ROOT"
ARGS="--no-cpu --steps 1 --warmup 0 --sweep-nodes 0 --sections c2_batch"
timeout -k 10 300 python -u bench.py $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- \
  python3 "$ROOT/bench.py" $ARGS > "$OUT/f.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- \
  python3 "$ROOT/bench.py" $ARGS > "$OUT/w.log" 2>&1
cd "$ROOT"
F=$(find "$OUT/fetch" -name "*counter_collection.csv" -print -quit)
W=$(find "$OUT/write" -name "*counter_collection.csv" -print -quit)
EV=$(python3 -c "import json;print(int(json.load(open('$OUT/bench.json'))['configs']['c2_batch']['roofline']['node_evals_per_launch']))")
python3 tools/pmc_traffic.py "$F" "$W" "k_chain" "$EV" 60 "$OUT/chain.json" > /dev/null
python3 tools/pmc_traffic.py "$F" "$W" "k_base" "$EV" 60 "$OUT/base.json" > /dev/null
python3 - "$OUT" "$EV" <<'PY'
import json, sys
out, ev = sys.argv[1], int(sys.argv[2])
c = json.load(open(out + "/chain.json"))
b = json.load(open(out + "/base.json"))
t = {"kernel": "k_base + k_chain (batched)", "nodes": ev, "bytes_per_node": 60,
     "bytes_per_launch": c["bytes_per_launch"] + b["bytes_per_launch"],
     "k_chain_bytes": c["bytes_per_launch"], "k_base_bytes": b["bytes_per_launch"],
     "algorithmic_bytes_per_launch": ev * 60, "correction": c["correction"]}
t["traffic_over_algorithmic"] = t["bytes_per_launch"] / t["algorithmic_bytes_per_launch"]
open(out + "/c2_batch_traffic.json", "w").write(json.dumps(t, indent=1) + "\n")
print(json.dumps(t, indent=1))
PY
