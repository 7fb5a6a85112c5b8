#!/bin/bash
# round 6: verification after the transform change -- GPU suite, smoke,
# bench (with the CPU leg), kernel trace of the bench command
set -e
tag=r16n
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 1200 $o/gpu_tests.log python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread
$chk 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
$chk 500 $o/bench.log python bench.py
grep "^{" $o/bench.log > $o/bench.json || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$chk 400 $o/prof.log rocprofv3 --kernel-trace --stats -d $PWD/$o/prof -o b --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline --no-secondary
python3 tools/rocpd_stats.py $(find $PWD/$o/prof -name "*kernel_trace.csv" | head -1) --top 70 > $o/rocprof_extract.txt
tail -3 $o/gpu_tests.log; grep smoke $o/smoke.log
python3 -c "import json; d=json.loads(open('$o/bench.json').read().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d.get('cpu_baseline',{}).get('value'), {k: (v.get('value'), v.get('roofline',{}).get('frac')) for k, v in d.get('secondary_workloads', {}).items()})"
head -8 $o/rocprof_extract.txt
exit 0
