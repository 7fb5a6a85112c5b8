set -e
timeout -k 10 300 python -u -m pytest tests/test_desc_grad.py tests/test_bb_train.py tests/test_gpu_correlation.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/wb_tests.log 2>&1
timeout -k 10 300 python bench.py --workload train_desc --steps 5 --warmup 2 > gpurun_out/bench_desc.json 2> gpurun_out/bench_desc.err
POSFEAT_WINPATCH=0 timeout -k 10 300 python bench.py --workload train_desc --steps 5 --warmup 2 > gpurun_out/bench_desc_taps.json 2>> gpurun_out/bench_desc.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_desc -o d -- python3 bench.py --workload train_desc --steps 3 --warmup 1 > gpurun_out/prof_desc.log 2>&1
