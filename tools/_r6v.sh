set -e
ab() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r6v_$tag.json 2>/dev/null; }
ab d1 POSFEAT_X=0
ab e1 POSFEAT_WINO_ENC=123
ab d2 POSFEAT_X=0
ab e2 POSFEAT_WINO_ENC=123
exit 0
