#!/bin/bash
# Round 3 GPU check: network preemption KATs + system caller + multi-device +
# eligibility parity, then the C4 k_system profile (stats, FETCH/WRITE passes).
set -eo pipefail
mkdir -p gpurun_out/r03e
timeout -k 10 700 python -u -m pytest tests/test_preemption.py tests/test_system_dropin.py tests/test_multi_device.py \
  tests/test_eligibility.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03e/pytest.log 2>&1
tail -3 gpurun_out/r03e/pytest.log
PE_API_PROF=1 timeout -k 10 120 python -u tools/c4_probe.py > gpurun_out/r03e/c4_probe.txt 2>&1
tail -30 gpurun_out/r03e/c4_probe.txt
bash tools/c4_pmc.sh
