set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/u4w_tests.log 2>&1 || true
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/bench_u4w.json 2> gpurun_out/bench_u4w.err
POSFEAT_UP4WINO=0 timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/bench_u4p.json 2>> gpurun_out/bench_u4w.err
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_u4w.log 2>&1
