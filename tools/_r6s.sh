set -e
# final measurement pass of the session (B=32 default): bench line with the
# CPU leg, kernel trace of the same command, PMC traffic of the dominant GEMM
# dispatches (600x36 blocks: the Winograd F(4x4) GEMMs of upconv2 / iconv2),
# and the training / correlation workloads
timeout -k 10 400 python bench.py > gpurun_out/bench_r6s.json 2> gpurun_out/bench_r6s.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6s -o b --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/prof_r6s.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  tag=$(echo $c | tr A-Z a-z | cut -d_ -f1)
  timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/pmc_r6s/$tag -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline > gpurun_out/pmc_r6s_$tag.log 2>&1
done
timeout -k 10 300 python bench.py --workload train_kp --no-cpu-baseline --steps 10 > gpurun_out/bench_train_kp_r6s.json 2>/dev/null
timeout -k 10 300 python bench.py --workload train_desc --no-cpu-baseline --steps 10 > gpurun_out/bench_train_desc_r6s.json 2>/dev/null
timeout -k 10 300 python bench.py --workload corr --no-cpu-baseline --steps 20 > gpurun_out/bench_corr_r6s.json 2>/dev/null
exit 0
