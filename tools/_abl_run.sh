set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_corr -o c -- python3 tools/bench_correlation.py 8 5 > gpurun_out/prof_corr.log 2>&1
