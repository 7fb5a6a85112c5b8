#!/bin/bash
# round 5: BatchNorm forward statistics from the conv epilogue: training tests, bench, A/B against the statistics pass
set -o pipefail
mkdir -p gpurun_out/r14f
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_bb_train.py tests/test_gpu_train_fullsize.py tests/test_gpu_syncbn.py \
  tests/test_gpu_trainer_plugpoints.py > gpurun_out/r14f/tests.txt 2>&1 || { tail -30 gpurun_out/r14f/tests.txt; exit 1; }
tail -2 gpurun_out/r14f/tests.txt
td() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r14f/td_$tag.txt 2>&1 || { tail -20 gpurun_out/r14f/td_$tag.txt; return 1; }
  grep '^{"metric' gpurun_out/r14f/td_$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['breakdown_ms'])"
}
td ship1 || exit 1
td ab_epi0 POSFEAT_HIP_LIB=posfeat_amd/libposfeat_hip_ab.so POSFEAT_TRAIN_BN_EPI=0 || exit 1
td ab_epi1 POSFEAT_HIP_LIB=posfeat_amd/libposfeat_hip_ab.so || exit 1
td ship2 || exit 1
