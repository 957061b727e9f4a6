#!/bin/bash
# the whole GPU suite
mkdir -p gpurun_out/r6k
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6k/gpu_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r6k/gpu_pytest.log
exit $rc
