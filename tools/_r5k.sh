set -e
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r5k.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r5k.json 2>/dev/null
timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/layer_timing_b32_r5k.txt 2>&1
exit 0
