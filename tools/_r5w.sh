set -e
# side-stream priority / width A/B at B=32 (same box)
ab() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r5w_$tag.json 2>/dev/null; }
ab d1 POSFEAT_X=0
ab p1 POSFEAT_SIDE_PRIO=1
ab p1g256 POSFEAT_SIDE_PRIO=1 POSFEAT_GFUSE_BLOCKS=256
ab p1g512 POSFEAT_SIDE_PRIO=1 POSFEAT_GFUSE_BLOCKS=512
ab d2 POSFEAT_X=0
ab p1b POSFEAT_SIDE_PRIO=1
exit 0
