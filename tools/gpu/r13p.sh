# round 5: F(6x6) on the encoder's layer2 / layer3 conv2 too (POSFEAT_WINO6_ENC
# A/B: "" = decoder + head only, "23" default): model tests, same-box bench pairs
set -o pipefail
mkdir -p gpurun_out/r13p
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bf6r.py tests/test_gpu_model.py tests/test_gpu_api.py > gpurun_out/r13p/tests.txt 2>&1 || { tail -30 gpurun_out/r13p/tests.txt; exit 1; }
tail -2 gpurun_out/r13p/tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
for i in 1 2; do for arm in 23 3 0; do
  POSFEAT_HIP_LIB=$PWD/posfeat_amd/libposfeat_hip_ab.so POSFEAT_WINO6_ENC=$arm timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/r13p/bench_enc_${arm}_$i.txt 2>&1 || { tail -20 gpurun_out/r13p/bench_enc_${arm}_$i.txt; exit 1; }
  grep '^{"metric' gpurun_out/r13p/bench_enc_${arm}_$i.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('enc=$arm', d['value'])"
done; done
# training decoder on F(6x6) (A/B): fixture error, fixture tests, speed
export POSFEAT_HIP_LIB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for arm in 0 1; do
  POSFEAT_TRAIN_WINO6=$arm timeout -k 10 300 python -u tools/bb_step_err.py > gpurun_out/r13p/err_w6_$arm.txt 2>&1 || { tail -20 gpurun_out/r13p/err_w6_$arm.txt; exit 1; }
  tail -3 gpurun_out/r13p/err_w6_$arm.txt
done
POSFEAT_TRAIN_WINO6=1 timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_bb_train.py tests/test_gpu_train_fullsize.py > gpurun_out/r13p/tests_train_w6.txt 2>&1; echo "train tests (wino6) rc=$?"; tail -3 gpurun_out/r13p/tests_train_w6.txt
for i in 1 2; do for arm in 0 1; do
  POSFEAT_TRAIN_WINO6=$arm timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r13p/td_w6_${arm}_$i.txt 2>&1 || { tail -20 gpurun_out/r13p/td_w6_${arm}_$i.txt; exit 1; }
  grep '^{"metric' gpurun_out/r13p/td_w6_${arm}_$i.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('train wino6=$arm', d['value'], d['breakdown_ms'])"
done; done
