#!/bin/bash
# same-box A/B of the C1 section: the session's start (9caa00e) vs now
mkdir -p gpurun_out/r6l
for k in 1 2 3; do
  PE_ENGINE_LIB=$PWD/abold/libnomadpe_9caa00e.so timeout -k 10 200 python bench.py --no-cpu --sections c1 > gpurun_out/r6l/old$k.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --no-cpu --sections c1 > gpurun_out/r6l/new$k.json 2>/dev/null || exit 1
done
for f in gpurun_out/r6l/*.json; do python3 -c "
import json,sys
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l)
print('$f', d['configs']['c1']['ms_per_eval'], d['ms_per_step'])"; done
