mkdir -p gpurun_out/r6b
B="python bench.py --steps 2 --warmup 1 --no-cpu --sweep-nodes 0 --sections c3_sharded,c3_sharded_1m,multi_loopback"
PE_FULL_PROF=1 timeout -k 10 120 python tools/c3_full_prof.py > gpurun_out/r6b/c3prof.txt 2>&1 && \
timeout -k 10 200 $B > gpurun_out/r6b/none.json 2>/dev/null && \
PE_SHARD_MERGE_ONE=1 timeout -k 10 200 $B > gpurun_out/r6b/launch.json 2>/dev/null && \
PE_SHARD_MERGE_ONE=1 PE_SHARD_MERGE=fused timeout -k 10 200 $B > gpurun_out/r6b/fused.json 2>/dev/null
