set -e
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r6x.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6x.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_r6x.json 2> gpurun_out/bench_r6x.err
exit 0
