set -e
timeout -k 10 900 python -u -m pytest tests/test_gpu_bf6r.py tests/test_gpu_model.py tests/test_gpu_bench_config.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/gpu_tests_r3y.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 > gpurun_out/bench_r3y.json 2>/dev/null
POSFEAT_UP2FUSE=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 > gpurun_out/bench_r3y_off.json 2>/dev/null
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r3y.log 2>&1
