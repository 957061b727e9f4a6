#!/bin/bash
# HBM traffic of the headline evaluation's device work (k_base + k_chain, the
# bench line's roofline kernel): FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes over the default bench loop, combined per evaluation by
# tools/pmc_traffic.py with the per-pattern FETCH_SIZE factors measured by
# tools/fetch_calib.hip (profiles/r04/fetch_calib_10000.json: k_base gathers
# 64-B records, counted 0.927 of their bytes -> x 1.079; k_chain reads 8-B
# values by position, counted 0.628 -> x 1.592). Writes
# gpurun_out/headline_pmc/headline_traffic.json.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/headline_pmc
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 3 --warmup 0 --sweep-nodes 0 --sections "" > "$OUT/f.json" 2> "$OUT/f.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 3 --warmup 0 --sweep-nodes 0 --sections "" > "$OUT/w.json" 2> "$OUT/w.err"
cd "$ROOT"
F=$(find "$OUT/fetch" -name "*counter_collection.csv" -print -quit)
W=$(find "$OUT/write" -name "*counter_collection.csv" -print -quit)
EV=$(python3 -c "import json;print(int(json.load(open('$OUT/f.json'))['roofline']['node_evals_per_launch']))")
python3 tools/pmc_traffic.py "$F" "$W" "k_chain" "$EV" 60 "$OUT/chain.json" 1.592 > /dev/null
python3 tools/pmc_traffic.py "$F" "$W" "k_base" 10000 60 "$OUT/base.json" 1.079 > /dev/null
python3 - "$OUT" "$EV" <<'PY'
import json, sys
out, ev = sys.argv[1], int(sys.argv[2])
c = json.load(open(out + "/chain.json"))
b = json.load(open(out + "/base.json"))
t = {"kernel": "k_base + k_chain", "node_evals": ev, "bytes_per_node_eval": 60,
     "bytes_per_launch": c["bytes_per_launch"] + b["bytes_per_launch"],
     "k_chain_bytes": c["bytes_per_launch"], "k_base_bytes": b["bytes_per_launch"],
     "algorithmic_bytes_per_launch": ev * 60,
     "dispatches": [c["dispatches"], b["dispatches"]],
     "k_chain_fetch_factor": c["fetch_factor"], "k_base_fetch_factor": b["fetch_factor"],
     "correction": "FETCH_SIZE x factor calibrated per access pattern (tools/fetch_calib.hip, "
                   "profiles/r04/fetch_calib_10000.json), WRITE_SIZE as is"}
t["traffic_over_algorithmic"] = t["bytes_per_launch"] / t["algorithmic_bytes_per_launch"]
open(out + "/headline_traffic.json", "w").write(json.dumps(t, indent=1) + "\n")
print(json.dumps(t, indent=1))
PY
