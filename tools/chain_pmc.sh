set -eo pipefail
ROOT=$GRAFT_REPO_ROOT; OUT=$ROOT/gpurun_out/chainpmc; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/chain_fetch" -o fetch -- python3 "$ROOT/bench.py" --no-cpu --steps 2 --warmup 0 --sweep-nodes 0 --sections "" > "$OUT/f.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/chain_write" -o write -- python3 "$ROOT/bench.py" --no-cpu --steps 2 --warmup 0 --sweep-nodes 0 --sections "" > "$OUT/w.log" 2>&1
cd $ROOT
EV=${EV:?set EV to roofline.node_evals_per_launch of the bench line}
python3 tools/pmc_traffic.py $(find $OUT/chain_fetch -name "*counter_collection.csv") $(find $OUT/chain_write -name "*counter_collection.csv") k_chain $EV 60 $OUT/chain_traffic.json
