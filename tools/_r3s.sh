export POSFEAT_WINO_ENC=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_config.py tests/test_gpu_precision.py tests/test_gpu_api.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3s.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 > gpurun_out/bench_r3s.json 2>gpurun_out/bench_r3s.err
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r3s.log 2>&1
unset POSFEAT_WINO_ENC
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 > gpurun_out/bench_r3s_off.json 2>/dev/null
exit 0
