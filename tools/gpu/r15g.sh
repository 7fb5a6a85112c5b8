#!/bin/bash
# after the weight-gradient knob commit (shipped behaviour unchanged): training + Winograd tests, smoke, bench
set -o pipefail
o=gpurun_out/r15g; mkdir -p $o
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_bb_train.py tests/test_gpu_train_fullsize.py tests/test_gpu_syncbn.py \
  tests/test_gpu_trainer_plugpoints.py tests/test_train_kp.py > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { tail -20 $o/smoke.txt; exit 1; }
grep smoke $o/smoke.txt
timeout -k 10 400 python bench.py > $o/bench.txt 2>&1 || { tail -20 $o/bench.txt; exit 1; }
grep '^{' $o/bench.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], {k: v.get('value') for k, v in d.get('secondary_workloads', {}).items()})"
