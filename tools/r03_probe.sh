#!/bin/bash
# Headline latency probes: k_chain per-step clocks (PE_CHAIN_PROF) on the C2
# workload, the drop-in phase split (PE_API_PROF), and the C5 loop split
# (PE_PLACE_PROF). Outputs in gpurun_out/$1/ (default probe).
set -eo pipefail
TAG=${1:-probe}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 120 python -u tools/chain_prof.py > "$OUT/chain_prof.txt" 2>&1 || { tail -30 "$OUT/chain_prof.txt"; exit 1; }
cat "$OUT/chain_prof.txt"
PE_API_PROF=1 timeout -k 10 120 python -u tools/dropin_probe.py > "$OUT/dropin_probe.txt" 2>&1 || { tail -30 "$OUT/dropin_probe.txt"; exit 1; }
tail -40 "$OUT/dropin_probe.txt"
PE_PLACE_PROF=1 timeout -k 10 180 python -u tools/c5_prof.py > "$OUT/c5_prof.txt" 2>&1 || { tail -30 "$OUT/c5_prof.txt"; exit 1; }
cat "$OUT/c5_prof.txt"
PE_API_PROF=1 timeout -k 10 120 python -u tools/dropin_probe.py 100 10 2000 > "$OUT/dropin_probe_c1.txt" 2>&1 || { tail -30 "$OUT/dropin_probe_c1.txt"; exit 1; }
tail -40 "$OUT/dropin_probe_c1.txt"
