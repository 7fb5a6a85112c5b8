#!/bin/bash
# round 6, first call: training tile-DB entries, training tests on the
# default plan, gcombine store ablation (A/B build), baseline bench line
set -e
tag=r16a
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 300 $o/tile_db_train.log python -u tools/tile_db.py --train $o/tile_db.txt
$chk 600 $o/train_tests.log python -u -m pytest tests/test_bb_train.py tests/test_gpu_train_fullsize.py tests/test_gpu_syncbn.py -m gpu -x -q --timeout 300 --timeout-method thread
POSFEAT_HIP_LIB=$PWD/posfeat_amd/libposfeat_hip_ab.so $chk 200 $o/lt_ab_default.log python -u tools/layer_timing.py 32
POSFEAT_HIP_LIB=$PWD/posfeat_amd/libposfeat_hip_ab.so POSFEAT_GC_NOSTORE=1 $chk 200 $o/lt_ab_nostore.log python -u tools/layer_timing.py 32
$chk 400 $o/bench.log python bench.py --no-cpu-baseline
grep "^{" $o/bench.log > $o/bench.json || true
tail -3 $o/train_tests.log; tail -2 $o/tile_db_train.log
grep -E "gcombine|head_tail|main stream" $o/lt_ab_default.log $o/lt_ab_nostore.log
python3 -c "import json; d=json.loads(open('$o/bench.json').read().splitlines()[-1]); print(d['value'], d['roofline']['frac'], {k: (v.get('value'), v.get('roofline')) for k, v in d.get('secondary_workloads', {}).items()})"
exit 0
