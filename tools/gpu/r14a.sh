# round 5: l2norm backward with the cell coordinates prefetched: corr tests, corr profile
set -o pipefail
mkdir -p gpurun_out/r14a
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_correlation.py tests/test_gpu_repeat.py > gpurun_out/r14a/tests.txt 2>&1 || { tail -30 gpurun_out/r14a/tests.txt; exit 1; }
tail -2 gpurun_out/r14a/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r14a/prof -o corr -- \
  python3 -u bench.py --workload corr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r14a/bench_corr.txt 2>&1 || exit 1
grep '^{"metric' gpurun_out/r14a/bench_corr.txt | cut -c1-160
for i in 1 2; do timeout -k 10 300 python3 -u bench.py --workload corr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r14a/corr_$i.txt 2>&1 || exit 1; grep '^{"metric' gpurun_out/r14a/corr_$i.txt | cut -c1-150; done
