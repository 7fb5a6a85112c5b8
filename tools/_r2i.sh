set -e
timeout -k 10 300 python bench.py --workload corr --steps 20 --warmup 3 > gpurun_out/bench_corr_r2i.json 2> gpurun_out/bench_corr_r2i.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_corr_r2i -o c --output-format csv -- python3 bench.py --workload corr --steps 10 --warmup 2 > gpurun_out/prof_corr_r2i.log 2>&1
