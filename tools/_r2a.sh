set -e
# round 2, first GPU pass: new parity tests + every GPU test, then the default bench line
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2a.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_r2a.json 2> gpurun_out/bench_r2a.err
