set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_config.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2e.log 2>&1
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r2e.log 2>&1
