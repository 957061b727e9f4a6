#!/bin/bash
# C4 host-overhead breakdown: the engine's API profile and a runtime timeline
mkdir -p gpurun_out/r6f
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PE_API_PROF=1 timeout -k 10 120 python tools/c4_probe.py > gpurun_out/r6f/probe.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
  -d gpurun_out/r6f/trace -o c4 -- python tools/c4_probe.py > gpurun_out/r6f/trace.txt 2>&1
rc=$?
tail -20 gpurun_out/r6f/probe.txt
exit $rc
