#!/bin/bash
# round 6: GPU suite + smoke on the final tree (after the alignment guards and
# fallbacks), then one bench line without the CPU leg
set -e
tag=r16zz7
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 1200 $o/gpu_tests.log python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread
tail -2 $o/gpu_tests.log
$chk 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
grep smoke $o/smoke.log
$chk 300 $o/bench.log python bench.py --no-cpu-baseline --no-secondary
grep "^{" $o/bench.log | cut -c1-200
exit 0
