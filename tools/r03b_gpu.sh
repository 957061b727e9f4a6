set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 600 python -u -m pytest tests/test_eligibility.py tests/test_system_dropin.py tests/test_shim_protocol.py tests/test_multi_device.py tests/test_dropin.py tests/test_c3_bench_size.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03b/pytest.log 2>&1; echo "pytest rc $?"; tail -40 gpurun_out/r03b/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --sweep-nodes 0 --sections c1,c4,c4_drop_in > gpurun_out/r03b/bench.json 2> gpurun_out/r03b/bench.err; echo "bench rc $?"
python -c "
import json;d=json.load(open('gpurun_out/r03b/bench.json'))
print('headline', d['value'], d['ms_per_step'], d.get('nodes_scored_per_s'))
for k,v in d['configs'].items(): print(k, {a:b for a,b in v.items() if a not in ('workload',)})
"
