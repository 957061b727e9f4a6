mkdir -p gpurun_out/r6c
PE_FULL_PROF=1 timeout -k 10 120 python tools/c3_full_prof.py > gpurun_out/r6c/c3prof.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_c3_bench_size.py tests/test_sweep_loop.py tests/test_engine_parity.py tests/test_wide_psets.py tests/test_distinct_property.py > gpurun_out/r6c/t.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 2 --warmup 1 --sweep-nodes 0 --sections c3 > gpurun_out/r6c/c3.json 2>/dev/null
