# round 5: 32-bit index splits (BN / Winograd transforms) + unrolled BN partials:
# parity tests, then a kernel-level profile of the descriptor training step
set -o pipefail
mkdir -p gpurun_out/r13g
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_model.py tests/test_gpu_train_fullsize.py tests/test_gpu_syncbn.py \
  tests/test_gpu_repeat.py tests/test_gpu_trainer_plugpoints.py \
  > gpurun_out/r13g/tests.txt 2>&1 || { tail -30 gpurun_out/r13g/tests.txt; exit 1; }
tail -3 gpurun_out/r13g/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r13g/prof -o td -- \
  python3 -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/r13g/bench_td.txt 2>&1 || { tail -20 gpurun_out/r13g/bench_td.txt; exit 1; }
tail -1 gpurun_out/r13g/bench_td.txt
f=$(ls gpurun_out/r13g/prof/*/td_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/r13g/td_kernel_stats.csv
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline \
  > gpurun_out/r13g/bench.txt 2>&1 || { tail -20 gpurun_out/r13g/bench.txt; exit 1; }
tail -1 gpurun_out/r13g/bench.txt | cut -c1-400
