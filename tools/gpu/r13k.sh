# round 5: training 3x3 stride-1 convs on bf16x6 halo tiles (A/B build,
# POSFEAT_TRAIN_HALO_BF6=1): fixture error vs fp64 and train_desc speed, both arms
set -o pipefail
mkdir -p gpurun_out/r13k
export PYTHONUNBUFFERED=1 POSFEAT_HIP_LIB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for arm in 0 1; do
  POSFEAT_TRAIN_HALO_BF6=$arm timeout -k 10 300 python -u tools/bb_step_err.py > gpurun_out/r13k/err_$arm.txt 2>&1 || { tail -20 gpurun_out/r13k/err_$arm.txt; exit 1; }
  tail -4 gpurun_out/r13k/err_$arm.txt
done
POSFEAT_TRAIN_HALO_BF6=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_bb_train.py > gpurun_out/r13k/tests_bf6.txt 2>&1; echo "bb_train tests (halo bf6) rc=$?"; tail -3 gpurun_out/r13k/tests_bf6.txt
for i in 1 2; do for arm in 0 1; do
  POSFEAT_TRAIN_HALO_BF6=$arm timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r13k/td_${arm}_$i.txt 2>&1 || { tail -20 gpurun_out/r13k/td_${arm}_$i.txt; exit 1; }
  grep '^{"metric' gpurun_out/r13k/td_${arm}_$i.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('arm $arm', d['value'], d['breakdown_ms'])"
done; done
