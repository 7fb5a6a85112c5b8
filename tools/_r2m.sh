set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_config.py tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2m.log 2>&1
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r2m.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r2m.json 2>/dev/null
timeout -k 10 400 python tools/extract_e2e.py --timing > gpurun_out/e2e_r2m_timing.json 2> gpurun_out/e2e_r2m_timing.err
timeout -k 10 400 python tools/extract_e2e.py > gpurun_out/e2e_r2m.json 2> gpurun_out/e2e_r2m.err
