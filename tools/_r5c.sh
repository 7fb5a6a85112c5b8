set -e
for b in 32 48 64; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --batch $b --steps 20 > gpurun_out/bench_r5c_b$b.json 2>/dev/null
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5c -o b --output-format csv -- python3 bench.py --batch 32 --steps 10 --no-cpu-baseline > gpurun_out/prof_r5c.log 2>&1
exit 0
