set -e
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r3e.json 2>/dev/null
POSFEAT_BF6B=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r3e_nob.json 2>/dev/null
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r3e2.json 2>/dev/null
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r3e.log 2>&1
