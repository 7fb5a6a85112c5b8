# round 5: extraction kernel profile (current build) + same-box train_desc A/B
# against the previous commit's library (abref/, built from cca2770)
set -o pipefail
mkdir -p gpurun_out/r13l
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r13l/prof -o ex -- \
  python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
  > gpurun_out/r13l/bench_ex.txt 2>&1 || { tail -20 gpurun_out/r13l/bench_ex.txt; exit 1; }
grep '^{"metric' gpurun_out/r13l/bench_ex.txt | cut -c1-160
for i in 1 2; do for arm in old new; do
  if [ $arm = old ]; then L=$PWD/abref/libposfeat_hip_cca2770.so; else L=$PWD/posfeat_amd/libposfeat_hip.so; fi
  POSFEAT_HIP_LIB=$L timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r13l/td_${arm}_$i.txt 2>&1 || { tail -20 gpurun_out/r13l/td_${arm}_$i.txt; exit 1; }
  grep '^{"metric' gpurun_out/r13l/td_${arm}_$i.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['value'], d['breakdown_ms'])"
done; done
