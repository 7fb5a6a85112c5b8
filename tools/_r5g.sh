set -e
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r5g.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r5g.json 2>/dev/null
POSFEAT_WINO_ENC=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r5g_enc0.json 2>/dev/null
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r5g_2.json 2>/dev/null
exit 0
