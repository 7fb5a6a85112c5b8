#!/bin/bash
# dgrad weight derivation writes the bf16 planes too: training tests, train_desc A/B against f4db0b4 (same box)
set -o pipefail
mkdir -p gpurun_out/r14u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_bb_train.py tests/test_gpu_train_fullsize.py tests/test_gpu_syncbn.py \
  tests/test_gpu_trainer_plugpoints.py > gpurun_out/r14u/tests.txt 2>&1 || { tail -30 gpurun_out/r14u/tests.txt; exit 1; }
tail -1 gpurun_out/r14u/tests.txt
REF=$PWD/abref/libposfeat_hip_f4db0b4.so
for i in 1 2; do
  for arm in new ref; do
    if [ $arm = ref ]; then L=$REF; else L=$PWD/posfeat_amd/libposfeat_hip.so; fi
    POSFEAT_HIP_LIB=$L timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r14u/td_${arm}$i.txt 2>&1 || { tail gpurun_out/r14u/td_${arm}$i.txt; exit 1; }
    grep '^{"metric' gpurun_out/r14u/td_${arm}$i.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm$i', d['value'], d['breakdown_ms'])"
  done
done
