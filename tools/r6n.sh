#!/bin/bash
mkdir -p gpurun_out/r6n
PE_API_PROF=1 timeout -k 10 300 python tools/c3_dropin_probe.py > gpurun_out/r6n/dropin.txt 2>&1 || exit 1
grep "per evaluation\|prepare_tg" gpurun_out/r6n/dropin.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_c3_bench_size.py \
  tests/test_engine_parity.py tests/test_wide_psets.py tests/test_distinct_property.py tests/test_metrics.py \
  tests/test_dropin.py tests/test_state_updates.py tests/test_eligibility.py > gpurun_out/r6n/t.log 2>&1
rc=$?
tail -2 gpurun_out/r6n/t.log
exit $rc
