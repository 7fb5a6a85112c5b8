set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_config.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r5d.log 2>&1
timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/layer_timing_b32_r5d.txt 2>&1
exit 0
