set -e
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3m.log 2>&1
timeout -k 10 300 python bench.py --steps 30 > gpurun_out/bench_r3m.json 2>gpurun_out/bench_r3m.err
timeout -k 10 300 python bench.py --workload train_desc --no-cpu-baseline --steps 10 > gpurun_out/bench_desc_r3m.json 2> gpurun_out/bench_desc_r3m.err
