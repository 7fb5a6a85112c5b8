set -e
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r5a.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_r5a.json 2> gpurun_out/bench_r5a.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5a -o run -- python bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_r5a_prof.json 2> gpurun_out/bench_r5a_prof.err
exit 0
