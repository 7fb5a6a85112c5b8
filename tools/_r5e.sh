set -e
# env A/B sweep of the extraction step at the new default batch (32)
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_r5e_$tag.json 2>/dev/null; }
run def0 POSFEAT_X=0
run noside POSFEAT_SIDE=0
run gb128 POSFEAT_GFUSE_BLOCKS=128
run gb256 POSFEAT_GFUSE_BLOCKS=256
run gb32 POSFEAT_GFUSE_BLOCKS=32
run at1 POSFEAT_SIDE_AT=1
run at3 POSFEAT_SIDE_AT=3
run winoenc POSFEAT_WINO_ENC=1
run def1 POSFEAT_X=0
exit 0
