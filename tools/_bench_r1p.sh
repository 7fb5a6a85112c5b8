set -e
# default bench line (with the CPU baseline) and the kernel trace of the same command
timeout -k 10 400 python bench.py > gpurun_out/bench_r1p.json 2> gpurun_out/bench_r1p.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_r1p -o b -- python3 bench.py --steps 5 --no-cpu-baseline > gpurun_out/prof_bench_r1p.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_desc_r1p -o d -- python3 bench.py --workload train_desc --steps 3 --warmup 1 > gpurun_out/prof_desc_r1p.log 2>&1
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r1p.log 2>&1
timeout -k 10 300 python bench.py --workload train_desc --steps 10 --warmup 3 > gpurun_out/bench_train_desc_r1p.json 2> gpurun_out/bench_train_desc_r1p.err
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_r1p.log 2>&1
