# same-box A/B of the headline (C2 drop-in, 20 steps) across the round-4, round-5 and current trees
mkdir -p gpurun_out/r6n
for i in 1 2; do
for t in tools/ab/r04 tools/ab/r05 .; do
  n=$(basename $(cd $t && pwd))
  (cd $t && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --sweep-nodes 0 --sections "" > /root/repo/gpurun_out/r6n/$n.$i.json 2>/dev/null) || exit 1
done
done
