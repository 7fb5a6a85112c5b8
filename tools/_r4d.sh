set -e
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4d.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 > gpurun_out/bench_r4d.json 2>/dev/null
