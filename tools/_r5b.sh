set -e
# batch sweep of the extraction step (images/s), same box
for b in 8 16 32 8; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --batch $b --steps 30 > gpurun_out/bench_r5b_b$b.json 2>/dev/null
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5b -o b --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/prof_r5b.log 2>&1
exit 0
