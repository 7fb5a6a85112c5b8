# round 5: Winograd F(6x6) for the extraction decoder + head.conv1: parity
# tests, smoke, bench (F6 default vs POSFEAT_WINO6=0 on the A/B build), profile
set -o pipefail
mkdir -p gpurun_out/r13m
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py -k "wino" > gpurun_out/r13m/tests_ops.txt 2>&1 || { tail -30 gpurun_out/r13m/tests_ops.txt; exit 1; }
grep -E "wino6 |passed|failed" gpurun_out/r13m/tests_ops.txt | tail -8
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_model.py tests/test_gpu_extract.py tests/test_gpu_api.py tests/test_gpu_repeat.py \
  > gpurun_out/r13m/tests.txt 2>&1 || { tail -30 gpurun_out/r13m/tests.txt; exit 1; }
tail -2 gpurun_out/r13m/tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
for i in 1 2; do for arm in 1 0; do
  POSFEAT_HIP_LIB=$PWD/posfeat_amd/libposfeat_hip_ab.so POSFEAT_WINO6=$arm timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/r13m/bench_w6_${arm}_$i.txt 2>&1 || { tail -20 gpurun_out/r13m/bench_w6_${arm}_$i.txt; exit 1; }
  grep '^{"metric' gpurun_out/r13m/bench_w6_${arm}_$i.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('wino6=$arm', d['value'], r['label'], r['avg_launch_ms'], r['frac'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r13m/prof -o ex -- \
  python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
  > gpurun_out/r13m/bench_ex.txt 2>&1 || { tail -20 gpurun_out/r13m/bench_ex.txt; exit 1; }
grep '^{"metric' gpurun_out/r13m/bench_ex.txt | cut -c1-120
