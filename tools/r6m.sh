mkdir -p gpurun_out/r6m
PE_API_PROF=1 timeout -k 10 120 python tools/c4_probe.py > gpurun_out/r6m/p.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r6m/t.log 2>&1
