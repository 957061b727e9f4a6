#!/bin/bash
# HBM traffic of the headline evaluation's k_base + k_chain with calibrated
# FETCH_SIZE factors (tools/fetch_calib.hip on the same box first): k_base
# gathers 64-byte node records through the visit order (the c_gather64<true>
# factor), k_chain reads 8-byte values by visit position (c_rows8). FETCH_SIZE
# and WRITE_SIZE in separate rocprofv3 passes. Writes
# gpurun_out/headline_pmc/{fetch_calib_10000,headline_traffic}.json.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/headline_pmc
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_f" -o f -- \
  "$ROOT/tools/fetch_calib" 10000 > "$OUT/calib.txt" 2> "$OUT/calib_f.err"
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib_w" -o w -- \
  "$ROOT/tools/fetch_calib" 10000 > /dev/null 2> "$OUT/calib_w.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 3 --warmup 0 --sweep-nodes 0 --sections "" > "$OUT/f.json" 2> "$OUT/f.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- \
  python3 "$ROOT/bench.py" --no-cpu --steps 3 --warmup 0 --sweep-nodes 0 --sections "" > "$OUT/w.json" 2> "$OUT/w.err"
cd "$ROOT"
python3 tools/fetch_calib.py $(find "$OUT/calib_f" -name "*counter_collection.csv" -print -quit) \
  $(find "$OUT/calib_w" -name "*counter_collection.csv" -print -quit) "$OUT/calib.txt" "$OUT/fetch_calib_10000.json" > /dev/null
F=$(find "$OUT/fetch" -name "*counter_collection.csv" -print -quit)
W=$(find "$OUT/write" -name "*counter_collection.csv" -print -quit)
EV=$(python3 -c "import json;print(int(json.load(open('$OUT/f.json'))['roofline']['node_evals_per_launch']))")
FB=$(python3 -c "import json;d=json.load(open('$OUT/fetch_calib_10000.json'))['patterns'];print(1.0/d['c_gather64<true>']['fetch_over_unique'])")
FC=$(python3 -c "import json;d=json.load(open('$OUT/fetch_calib_10000.json'))['patterns'];print(1.0/d['c_rows8']['fetch_over_unique'])")
python3 tools/pmc_traffic.py "$F" "$W" "k_chain" "$EV" 60 "$OUT/chain.json" "$FC" > /dev/null
python3 tools/pmc_traffic.py "$F" "$W" "k_base" 10000 60 "$OUT/base.json" "$FB" > /dev/null
python3 - "$OUT" "$EV" <<'PY'
import json, sys
out, ev = sys.argv[1], int(sys.argv[2])
c = json.load(open(out + "/chain.json"))
b = json.load(open(out + "/base.json"))
t = {"kernel": "k_base + k_chain", "node_evals": ev, "bytes_per_node_eval": 60,
     "bytes_per_launch": c["bytes_per_launch"] + b["bytes_per_launch"],
     "k_chain_bytes": c["bytes_per_launch"], "k_base_bytes": b["bytes_per_launch"],
     "k_chain_fetch_factor": c["fetch_factor"], "k_base_fetch_factor": b["fetch_factor"],
     "bounds_bytes_per_launch": [c["fetch_counted_bytes_per_launch"] + b["fetch_counted_bytes_per_launch"]
                                 + c["write_bytes_per_launch"] + b["write_bytes_per_launch"],
                                 2 * (c["fetch_counted_bytes_per_launch"] + b["fetch_counted_bytes_per_launch"])
                                 + c["write_bytes_per_launch"] + b["write_bytes_per_launch"]],
     "algorithmic_bytes_per_launch": ev * 60,
     "dispatches": [c["dispatches"], b["dispatches"]],
     "correction": "FETCH_SIZE x factor calibrated per access pattern on this box (k_base: 64-B record "
                   "gathers, c_gather64<true>; k_chain: 8-B values by position, c_rows8), WRITE_SIZE as is; "
                   "bounds: FETCH_SIZE x 1 and x 2"}
t["traffic_over_algorithmic"] = t["bytes_per_launch"] / t["algorithmic_bytes_per_launch"]
open(out + "/headline_traffic.json", "w").write(json.dumps(t, indent=1) + "\n")
print(json.dumps(t, indent=1))
PY
