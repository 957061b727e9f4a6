#!/bin/bash
# multi-NIC parity and the network / preemption suites around it
mkdir -p gpurun_out/r6d
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_multi_nic.py tests/test_preemption.py tests/test_static_ports.py tests/test_metrics.py \
  tests/test_ploop.py tests/test_wide_eviction.py tests/test_engine_parity.py > gpurun_out/r6d/t.log 2>&1
rc=$?
tail -30 gpurun_out/r6d/t.log
exit $rc
