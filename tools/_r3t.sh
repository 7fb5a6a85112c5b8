set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_desc_r3t -o d -- python3 bench.py --workload train_desc --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_desc_r3t.log 2>&1
