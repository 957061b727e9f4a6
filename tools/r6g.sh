#!/bin/bash
mkdir -p gpurun_out/r6g
for k in 1 2 3; do
timeout -k 10 120 python tools/c4_probe.py 400 > gpurun_out/r6g/new$k.txt 2>&1 && \
PE_SYS_SPLIT_SYNC=1 timeout -k 10 120 python tools/c4_probe.py 400 > gpurun_out/r6g/old$k.txt 2>&1 || exit 1
done
for f in gpurun_out/r6g/new*.txt gpurun_out/r6g/old*.txt; do echo $f $(tail -1 $f); done
