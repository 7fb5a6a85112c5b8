set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_bench_config.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3a.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r3a.json 2>/dev/null
