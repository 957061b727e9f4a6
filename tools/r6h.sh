#!/bin/bash
# C3 service-wave loop: parity, then timing against k_fullpass_lds
mkdir -p gpurun_out/r6h
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_c3_bench_size.py tests/test_sweep_loop.py tests/test_engine_parity.py tests/test_spec_view.py \
  tests/test_dropin.py tests/test_metrics.py > gpurun_out/r6h/t.log 2>&1
rc=$?
tail -4 gpurun_out/r6h/t.log
[ $rc -ne 0 ] && exit $rc
for k in 1 2; do
timeout -k 10 120 python tools/c3_full_prof.py > gpurun_out/r6h/svc$k.txt 2>&1 && \
PE_FULL_SVC=0 timeout -k 10 120 python tools/c3_full_prof.py > gpurun_out/r6h/lds$k.txt 2>&1 || exit 1
done
for f in gpurun_out/r6h/svc*.txt gpurun_out/r6h/lds*.txt; do echo $f; tail -2 $f; done
timeout -k 10 300 python tools/c3_dropin_probe.py > gpurun_out/r6h/dropin.txt 2>&1; tail -5 gpurun_out/r6h/dropin.txt
