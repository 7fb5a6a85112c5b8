#!/bin/bash
# A/B: the train-mode decoder's Winograd GEMMs on the 16x16x32 bf6x tiles (POSFEAT_TRAIN_WINO_BF6X=1)
set -o pipefail
o=gpurun_out/r15i; mkdir -p $o
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
POSFEAT_HIP_LIB=$AB timeout -k 10 300 python -u tools/bb_step_err.py > $o/err_base.txt 2>&1 || { tail -20 $o/err_base.txt; exit 1; }
POSFEAT_HIP_LIB=$AB POSFEAT_TRAIN_WINO_BF6X=1 timeout -k 10 300 python -u tools/bb_step_err.py > $o/err_x.txt 2>&1 || { tail -20 $o/err_x.txt; exit 1; }
tail -4 $o/err_base.txt; tail -4 $o/err_x.txt
td() {  # tag env...
  local tag=$1; shift
  env POSFEAT_HIP_LIB=$AB "$@" timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline > $o/td_$tag.txt 2>&1 || { tail -20 $o/td_$tag.txt; return 1; }
  grep '^{"metric' $o/td_$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], {k: round(v, 2) for k, v in d['breakdown_ms'].items()} if isinstance(d.get('breakdown_ms'), dict) else '')"
}
td base || exit 1
td x POSFEAT_TRAIN_WINO_BF6X=1 || exit 1
td base2 || exit 1
td x2 POSFEAT_TRAIN_WINO_BF6X=1 || exit 1
POSFEAT_HIP_LIB=$AB POSFEAT_TRAIN_WINO_BF6X=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_bb_train.py tests/test_gpu_train_fullsize.py > $o/tests_x.txt 2>&1; tail -15 $o/tests_x.txt
exit 0
