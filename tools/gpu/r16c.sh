#!/bin/bash
# round 6: full GPU suite after the hazard-guard changes (no packed fp32 in 14
# kernels, lgkmcnt(0) before the bf6d/bf6s K-loop barriers), smoke, bench
set -e
tag=r16c
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 1200 $o/gpu_tests.log python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread
$chk 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
$chk 400 $o/bench.log python bench.py --no-cpu-baseline
grep "^{" $o/bench.log > $o/bench.json || true
$chk 200 $o/lt.log python -u tools/layer_timing.py 32
tail -4 $o/gpu_tests.log; grep smoke $o/smoke.log
grep -E "largest relative errors vs fp64 \(err" $o/gpu_tests.log | tail -2
python3 -c "import json; d=json.loads(open('$o/bench.json').read().splitlines()[-1]); print(d['value'], d['roofline']['frac'], {k: (v.get('value'), v.get('roofline',{}).get('frac')) for k, v in d.get('secondary_workloads', {}).items()})"
exit 0
