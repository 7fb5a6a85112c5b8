set -e
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3u.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 > gpurun_out/bench_r3u.json 2>/dev/null
timeout -k 10 300 python bench.py --workload train_desc --no-cpu-baseline --steps 10 > gpurun_out/bench_desc_r3u.json 2>/dev/null
timeout -k 10 300 python bench.py --workload train_kp --no-cpu-baseline --steps 10 > gpurun_out/bench_kp_r3u.json 2>/dev/null
