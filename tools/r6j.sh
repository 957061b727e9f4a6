#!/bin/bash
mkdir -p gpurun_out/r6j
PE_SVC_PROF=1 timeout -k 10 120 python tools/c3_full_prof.py > gpurun_out/r6j/a.txt 2>&1 && \
timeout -k 10 120 python tools/c3_full_prof.py > gpurun_out/r6j/b.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_c3_bench_size.py tests/test_engine_parity.py > gpurun_out/r6j/t.log 2>&1
rc=$?
cat gpurun_out/r6j/a.txt; grep pe_place gpurun_out/r6j/b.txt; tail -n 2 gpurun_out/r6j/t.log
exit $rc
