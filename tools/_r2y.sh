set -e
POSFEAT_BF6=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_config.py tests/test_gpu_ops.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2y.log 2>&1 || true
POSFEAT_BF6=2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r2y_bf6p.json 2>gpurun_out/bench_r2y.err
POSFEAT_BF6=2 timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r2y_bf6p.log 2>&1
