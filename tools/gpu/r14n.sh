#!/bin/bash
# training direct convs on autotuned tiles: tests, A/B bench (POSFEAT_TRAIN_TUNE=0), per-label timing
set -o pipefail
mkdir -p gpurun_out/r14n
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_bb_train.py tests/test_gpu_train_fullsize.py tests/test_gpu_syncbn.py \
  tests/test_gpu_trainer_plugpoints.py -s > gpurun_out/r14n/tests.txt 2>&1 || { tail -40 gpurun_out/r14n/tests.txt; exit 1; }
grep -E "passed|failed|largest relative" gpurun_out/r14n/tests.txt | tail -5
td() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r14n/td_$tag.txt 2>&1 || { tail -20 gpurun_out/r14n/td_$tag.txt; return 1; }
  grep '^{"metric' gpurun_out/r14n/td_$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['breakdown_ms'])"
}
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
td ab_tune0 POSFEAT_HIP_LIB=$AB POSFEAT_TRAIN_TUNE=0 || exit 1
td ab_tune1 POSFEAT_HIP_LIB=$AB || exit 1
td ship || exit 1
timeout -k 10 300 python -u tools/train_layer_timing.py 8 > gpurun_out/r14n/tlt.txt 2>&1 || exit 1
head -40 gpurun_out/r14n/tlt.txt
