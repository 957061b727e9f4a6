#!/bin/bash
# lean service evaluation vs the generic one, then parity
mkdir -p gpurun_out/r6o
for k in 1 2; do
timeout -k 10 120 python tools/c3_full_prof.py > gpurun_out/r6o/lean$k.txt 2>&1 && \
PE_SVC_LEAN=0 timeout -k 10 120 python tools/c3_full_prof.py > gpurun_out/r6o/gen$k.txt 2>&1 || exit 1
done
grep -H pe_place gpurun_out/r6o/*.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_c3_bench_size.py \
  tests/test_engine_parity.py tests/test_sweep_loop.py tests/test_dropin.py tests/test_spec_view.py tests/test_metrics.py > gpurun_out/r6o/t.log 2>&1
rc=$?
tail -2 gpurun_out/r6o/t.log
exit $rc
