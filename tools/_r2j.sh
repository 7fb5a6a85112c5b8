set -e
timeout -k 10 900 python -u -m pytest tests/test_desc_grad.py tests/test_bb_train.py tests/test_gpu_correlation.py tests/test_gpu_matchers.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2j.log 2>&1
timeout -k 10 300 python bench.py --workload corr --steps 20 --warmup 3 > gpurun_out/bench_corr_r2j.json 2> gpurun_out/bench_corr_r2j.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_corr_r2j -o c --output-format csv -- python3 bench.py --workload corr --steps 10 --warmup 2 > gpurun_out/prof_corr_r2j.log 2>&1
