# DiskLoss WR pass: reinforce terms in fp32 per stage: corr tests, corr profile, bench
set -o pipefail
mkdir -p gpurun_out/r14s
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_correlation.py tests/test_gpu_repeat.py > gpurun_out/r14s/tests.txt 2>&1 || { tail -30 gpurun_out/r14s/tests.txt; exit 1; }
tail -2 gpurun_out/r14s/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r14s/prof -o corr -- \
  python3 -u bench.py --workload corr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r14s/bench_corr.txt 2>&1 || exit 1
grep '^{"metric' gpurun_out/r14s/bench_corr.txt | cut -c1-160
for i in 1 2; do timeout -k 10 300 python3 -u bench.py --workload corr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r14s/corr_$i.txt 2>&1 || exit 1; grep '^{"metric' gpurun_out/r14s/corr_$i.txt | cut -c1-150; done
python3 tools/rocpd_stats.py gpurun_out/r14s/prof/corr_results.db --top 12 > gpurun_out/r14s/rocprof_corr.txt 2>&1 || ls -R gpurun_out/r14s/prof | head
head -8 gpurun_out/r14s/rocprof_corr.txt
