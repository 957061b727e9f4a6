mkdir -p gpurun_out/r6o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_metrics.py tests/test_cores.py > gpurun_out/r6o/t.log 2>&1 ; \
PE_METRICS_PROF=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --sweep-nodes 0 --sections "" > gpurun_out/r6o/b.json 2> gpurun_out/r6o/b.err
