set -e
# round 3 measurement pass: bench line (with the CPU leg), kernel trace of the
# same command, PMC traffic of the dominant GEMM dispatch (150x36 blocks:
# the Winograd F(4x4) GEMMs of upconv2 / iconv2, conv_bf6b_kernel)
timeout -k 10 400 python bench.py > gpurun_out/bench_r3z.json 2> gpurun_out/bench_r3z.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3z -o b --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/prof_r3z.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  tag=$(echo $c | tr A-Z a-z | cut -d_ -f1)
  timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/pmc_r3z/$tag -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --timing-steps 1 --no-cpu-baseline > gpurun_out/pmc_r3z_$tag.log 2>&1
done
