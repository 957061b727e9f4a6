#!/bin/bash
# k_system two-phase (row-order evaluation + list-order gather) vs the scattered
# single pass: parity, the size sweep of both, then the PMC passes.
set -eo pipefail
mkdir -p gpurun_out/r03f
timeout -k 10 400 python -u -m pytest tests/test_system_dropin.py tests/test_preemption.py tests/test_engine_parity.py -m gpu -x -q \
  -k "system or System" --timeout 300 --timeout-method thread > gpurun_out/r03f/pytest.log 2>&1
tail -3 gpurun_out/r03f/pytest.log
timeout -k 10 200 python3 tools/c4_prof.py > gpurun_out/r03f/gather.jsonl 2>&1
PE_SYS_SCATTER=1 timeout -k 10 200 python3 tools/c4_prof.py > gpurun_out/r03f/scatter.jsonl 2>&1
cat gpurun_out/r03f/gather.jsonl gpurun_out/r03f/scatter.jsonl
bash tools/c4_pmc.sh
