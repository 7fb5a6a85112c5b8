#!/bin/bash
# full GPU suite + A/B-build tests + smoke + bench line after the training autotune
set -e
o=gpurun_out/r14o
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 900 $o/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
POSFEAT_HIP_LIB=$PWD/posfeat_amd/libposfeat_hip_ab.so $chk 600 $o/gpu_tests_ab.log python -u -m pytest tests/test_gpu_correlation.py tests/test_gpu_train_tap.py -m gpu -x -q -rs --timeout 300 --timeout-method thread
$chk 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
$chk 400 $o/bench.log python bench.py
grep "^{" $o/bench.log > $o/bench.json || true
tail -2 $o/gpu_tests.log; tail -1 $o/gpu_tests_ab.log; grep smoke $o/smoke.log
python3 -c "import json; d=json.loads(open('$o/bench.json').read().splitlines()[-1]); print(d['value'], d['roofline']['frac'], {k: v.get('value') for k, v in d.get('secondary_workloads', {}).items()})"
