set -e
POSFEAT_BF6=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2v_ops.log 2>&1 || true
POSFEAT_BF6=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_config.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2v_model.log 2>&1 || true
POSFEAT_BF6=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r2v_bf6.json 2>gpurun_out/bench_r2v_bf6.err
POSFEAT_BF6=1 timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r2v_bf6.log 2>&1
