#!/bin/bash
# eviction width 32 and the preemption suites around it
mkdir -p gpurun_out/r6e
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_wide_eviction.py tests/test_preemption.py tests/test_ploop.py tests/test_spec_view.py \
  tests/test_cores.py tests/test_multi_nic.py > gpurun_out/r6e/t.log 2>&1
rc=$?
tail -25 gpurun_out/r6e/t.log
exit $rc
