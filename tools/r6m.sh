#!/bin/bash
mkdir -p gpurun_out/r6m
PE_API_PROF=1 timeout -k 10 300 python tools/c3_dropin_probe.py > gpurun_out/r6m/dropin.txt 2>&1 || exit 1
grep "per evaluation\|prepare_tg" gpurun_out/r6m/dropin.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6m/gpu_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r6m/gpu_pytest.log
exit $rc
