mkdir -p gpurun_out/r6i
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_metrics.py tests/test_system_dropin.py tests/test_abi.py > gpurun_out/r6i/t.log 2>&1 ; \
PE_METRICS_PROF=1 timeout -k 10 400 python bench.py --steps 10 --warmup 2 --sweep-nodes 0 --sections c4_drop_in > gpurun_out/r6i/b.json 2> gpurun_out/r6i/b.err
