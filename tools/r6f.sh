mkdir -p gpurun_out/r6f
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_metrics.py -k "system" > gpurun_out/r6f/t.log 2>&1 ; \
PE_METRICS_PROF=1 timeout -k 10 600 python bench.py --steps 4 --warmup 1 --sweep-nodes 0 --sections c3,c4_drop_in,c5 --c5-cpu-seconds 30 > gpurun_out/r6f/b.json 2> gpurun_out/r6f/b.err
