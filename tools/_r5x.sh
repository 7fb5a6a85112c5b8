set -e
ab() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r5x_$tag.json 2>/dev/null; }
ab d1 POSFEAT_X=0
ab p1 POSFEAT_BF6B_PREF=1
ab d2 POSFEAT_X=0
ab p2 POSFEAT_BF6B_PREF=1
timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r5x_d.txt 2>&1
POSFEAT_BF6B_PREF=1 timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r5x_p.txt 2>&1
exit 0
