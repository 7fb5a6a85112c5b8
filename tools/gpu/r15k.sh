#!/bin/bash
# after restoring the 32x32x16 training decoder GEMMs as default: training tests, smoke
set -o pipefail
o=gpurun_out/r15k; mkdir -p $o
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_bb_train.py tests/test_gpu_train_fullsize.py tests/test_gpu_syncbn.py \
  tests/test_gpu_trainer_plugpoints.py tests/test_train_kp.py tests/test_gpu_bf6x.py > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { tail -20 $o/smoke.txt; exit 1; }
grep smoke $o/smoke.txt
timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline > $o/td.txt 2>&1 || { tail -20 $o/td.txt; exit 1; }
grep '^{"metric' $o/td.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])"
