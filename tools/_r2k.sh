set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_config.py tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2k.log 2>&1
POSFEAT_GLDS3=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2k_g3.log 2>&1
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r2k_g2.log 2>&1
POSFEAT_GLDS3=1 timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r2k_g3.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r2k_g2.json 2>/dev/null
POSFEAT_GLDS3=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r2k_g3.json 2>/dev/null
