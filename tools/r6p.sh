#!/bin/bash
mkdir -p gpurun_out/r6p
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_state_updates.py tests/test_dropin.py > gpurun_out/r6p/t2.log 2>&1
rc=$?
tail -2 gpurun_out/r6p/t2.log
exit $rc
