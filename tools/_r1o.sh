set -e
# up4 Winograd: smoke + GPU tests, bench line, kernel trace of the bench, PMC traffic passes
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_r1o.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_r1o.json 2> gpurun_out/bench_r1o.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_r1o -o b -- python3 bench.py --steps 5 --no-cpu-baseline > gpurun_out/prof_bench_r1o.log 2>&1
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r1o.log 2>&1
mkdir -p gpurun_out/pmc_r1o
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_r1o/fetch -o pmc --output-format csv -- python3 tools/layer_timing.py 8 480 640 > gpurun_out/pmc_r1o/fetch.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_r1o/write -o pmc --output-format csv -- python3 tools/layer_timing.py 8 480 640 > gpurun_out/pmc_r1o/write.log 2>&1
