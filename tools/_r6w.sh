set -e
ab() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r6w_$tag.json 2>/dev/null; }
ab g64a POSFEAT_X=0
ab g128a POSFEAT_GFUSE_BLOCKS=128
ab g32a POSFEAT_GFUSE_BLOCKS=32
ab g64b POSFEAT_X=0
ab g128b POSFEAT_GFUSE_BLOCKS=128
ab g32b POSFEAT_GFUSE_BLOCKS=32
exit 0
