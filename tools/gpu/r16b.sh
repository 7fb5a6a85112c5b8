#!/bin/bash
# round 6: multi-rank entry-point tests, tightened parity bounds (measured errors printed)
set -e
tag=r16b
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 900 $o/multirank.log python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v -s --timeout 600 --timeout-method thread
$chk 900 $o/bounds.log python -u -m pytest tests/test_gpu_model.py tests/test_gpu_api.py tests/test_gpu_precision.py tests/test_gpu_bench_config.py tests/test_gpu_train_fullsize.py -m gpu -v -s --timeout 600 --timeout-method thread
$chk 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
grep -E "passed|failed|error" $o/multirank.log | tail -3
grep -E "passed|failed" $o/bounds.log | tail -3
grep -E "max abs err|largest|relative L2|smoke ok" $o/*.log | sort -t'(' -k3 | tail -40
exit 0
