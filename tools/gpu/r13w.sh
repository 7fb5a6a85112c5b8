# round 5: the forward F(6x6) V kept for the weight gradient: training tests, profile, bench

set -o pipefail
mkdir -p gpurun_out/r13w
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_bb_train.py tests/test_gpu_train_fullsize.py tests/test_gpu_syncbn.py \
  tests/test_gpu_trainer_plugpoints.py > gpurun_out/r13w/tests.txt 2>&1 || { tail -30 gpurun_out/r13w/tests.txt; exit 1; }
tail -2 gpurun_out/r13w/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r13w/prof -o td -- \
  python3 -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/r13w/bench_td.txt 2>&1 || { tail -20 gpurun_out/r13w/bench_td.txt; exit 1; }
grep '^{"metric' gpurun_out/r13w/bench_td.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['breakdown_ms'])"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r13w/td_$i.txt 2>&1 || exit 1
  grep '^{"metric' gpurun_out/r13w/td_$i.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['breakdown_ms'])"
done
