set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/side_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/bench_side.json 2> gpurun_out/bench_side.err
POSFEAT_SIDE=0 timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/bench_noside.json 2>> gpurun_out/bench_side.err
