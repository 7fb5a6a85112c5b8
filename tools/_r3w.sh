set -e
for cfg in "POSFEAT_GFUSE_BLOCKS=64" "POSFEAT_GFUSE_BLOCKS=32" "POSFEAT_GFUSE_BLOCKS=48" "POSFEAT_GFUSE_BLOCKS=96" "POSFEAT_GFUSE_BLOCKS=64 POSFEAT_SIDE_AT=1" "POSFEAT_GFUSE_BLOCKS=32 POSFEAT_SIDE_AT=1" "POSFEAT_GFUSE_BLOCKS=512"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 > "gpurun_out/bench_r3w2_${cfg// /_}.json" 2>/dev/null
done
