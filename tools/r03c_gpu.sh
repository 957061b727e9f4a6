set -o pipefail
mkdir -p gpurun_out/r03c
timeout -k 10 600 python -u -m pytest tests/test_system_dropin.py tests/test_multi_device.py tests/test_full_size.py tests/test_engine_parity.py tests/test_eligibility.py -m gpu -q --timeout 300 --timeout-method thread -k "system or c4 or System or multi or split or full" > gpurun_out/r03c/pytest.log 2>&1; echo "pytest rc $?"; tail -15 gpurun_out/r03c/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --sweep-nodes 0 --sections c4,c4_drop_in > gpurun_out/r03c/bench.json 2> gpurun_out/r03c/bench.err; echo "bench rc $?"
python -c "
import json;d=json.load(open('gpurun_out/r03c/bench.json'))
for k,v in d['configs'].items(): print(k, {a:b for a,b in v.items() if a not in ('workload',)})
"
bash tools/c4_pmc.sh
