# round 5: F(6x6) weight gradient for the train-mode decoder (A/B POSFEAT_TRAIN_WINO6_WGRAD): training tests, fixture error, speed

set -o pipefail
mkdir -p gpurun_out/r13t
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_bb_train.py tests/test_gpu_train_fullsize.py tests/test_gpu_syncbn.py \
  tests/test_gpu_trainer_plugpoints.py > gpurun_out/r13t/tests.txt 2>&1 || { tail -30 gpurun_out/r13t/tests.txt; exit 1; }
tail -2 gpurun_out/r13t/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r13t/prof -o td -- \
  python3 -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/r13t/bench_td.txt 2>&1 || { tail -20 gpurun_out/r13t/bench_td.txt; exit 1; }
grep '^{"metric' gpurun_out/r13t/bench_td.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['breakdown_ms'])"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r13t/td_$i.txt 2>&1 || exit 1
  grep '^{"metric' gpurun_out/r13t/td_$i.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['breakdown_ms'])"
done
export POSFEAT_HIP_LIB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for arm in 0 1; do
  POSFEAT_TRAIN_WINO6_WGRAD=$arm timeout -k 10 300 python -u tools/bb_step_err.py > gpurun_out/r13t/err_wg_$arm.txt 2>&1 || { tail -20 gpurun_out/r13t/err_wg_$arm.txt; exit 1; }
  tail -3 gpurun_out/r13t/err_wg_$arm.txt
done
for i in 1 2; do for arm in 0 1; do
  POSFEAT_TRAIN_WINO6_WGRAD=$arm timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r13t/td_wg_${arm}_$i.txt 2>&1 || exit 1
  grep '^{"metric' gpurun_out/r13t/td_wg_${arm}_$i.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('wgrad6=$arm', d['value'], d['breakdown_ms'])"
done; done
# DiskLoss SUM-pass epilogue (fewer VALU): correlation tests (flash == dense A/B,
# vs reference), repeat test, corr bench
unset POSFEAT_HIP_LIB
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_correlation.py tests/test_gpu_repeat.py > gpurun_out/r13t/tests_corr.txt 2>&1 || { tail -30 gpurun_out/r13t/tests_corr.txt; exit 1; }
tail -2 gpurun_out/r13t/tests_corr.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r13t/prof_corr -o corr -- \
  python3 -u bench.py --workload corr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r13t/bench_corr.txt 2>&1 || exit 1
grep '^{"metric' gpurun_out/r13t/bench_corr.txt | cut -c1-200
