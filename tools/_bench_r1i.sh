set -e
# default bench line (with the CPU baseline) and the kernel trace of the same command
timeout -k 10 400 python bench.py > gpurun_out/bench_r1i.json 2> gpurun_out/bench_r1i.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_r1i -o b -- python3 bench.py --steps 5 --no-cpu-baseline > gpurun_out/prof_bench_r1i.log 2>&1
