set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_tap.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r5h_tap.log 2>&1 || true
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r5h.log 2>&1 || true
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r5h.json 2>/dev/null
POSFEAT_WINO_ENC=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r5h_enc0.json 2>/dev/null
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r5h_2.json 2>/dev/null
exit 0
