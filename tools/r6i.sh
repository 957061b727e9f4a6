#!/bin/bash
mkdir -p gpurun_out/r6i
timeout -k 10 120 python tools/c3_full_prof.py > gpurun_out/r6i/svc.txt 2>&1 && \
PE_API_PROF=1 timeout -k 10 300 python tools/c3_dropin_probe.py > gpurun_out/r6i/dropin.txt 2>&1
rc=$?
tail -2 gpurun_out/r6i/svc.txt; cat gpurun_out/r6i/dropin.txt | tail -45
exit $rc
