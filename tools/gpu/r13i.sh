# round 5: PMC wave-state / instruction-mix passes over the descriptor training
# step (wgrad kernels), then the f3 extraction runs (tile database, staged reader)
set -o pipefail
mkdir -p gpurun_out/r13i
export PYTHONUNBUFFERED=1
BENCH_ARGS="--workload train_desc --steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline" \
  bash tools/pmc_kernels.sh gpurun_out/r13i/pmc || { echo pmc failed; exit 1; }
grep -h "rc=" gpurun_out/r13i/pmc/*.log
sed -i 's#gpurun_out/r13f#gpurun_out/r13i#g' tools/gpu/r13f.sh
bash tools/gpu/r13f.sh
