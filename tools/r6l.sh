mkdir -p gpurun_out/r6l
PE_API_PROF=1 timeout -k 10 120 python tools/c4_probe.py > gpurun_out/r6l/p.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_system_dropin.py tests/test_shard.py tests/test_full_size.py tests/test_metrics.py -k "system or c4 or shard" > gpurun_out/r6l/t.log 2>&1
