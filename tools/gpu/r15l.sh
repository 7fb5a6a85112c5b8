#!/bin/bash
# round 5 final verification: GPU suite (+ A/B-build tests), smoke, bench line, kernel traces of extract and train_desc
set -e
tag=r15l
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 900 $o/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
POSFEAT_HIP_LIB=$PWD/posfeat_amd/libposfeat_hip_ab.so $chk 600 $o/gpu_tests_ab.log python -u -m pytest tests/test_gpu_correlation.py tests/test_gpu_train_tap.py -m gpu -x -q -rs --timeout 300 --timeout-method thread
$chk 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
$chk 400 $o/bench.log python bench.py
grep "^{" $o/bench.log > $o/bench.json || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$chk 400 $o/prof.log rocprofv3 --kernel-trace --stats -d $PWD/$o/prof -o b --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline --no-secondary
$chk 400 $o/prof_td.log rocprofv3 --kernel-trace --stats -d $PWD/$o/proftd -o td --output-format csv -- python3 bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline
python3 tools/rocpd_stats.py $(find $PWD/$o/prof -name "*kernel_trace.csv" | head -1) --top 60 > $o/rocprof_extract.txt
python3 tools/rocpd_stats.py $(find $PWD/$o/proftd -name "*kernel_trace.csv" | head -1) --top 60 > $o/rocprof_train_desc.txt
tail -3 $o/gpu_tests.log; tail -2 $o/gpu_tests_ab.log; cat $o/smoke.log | grep smoke
python3 -c "import json; d=json.loads(open('$o/bench.json').read().splitlines()[-1]); print(d['value'], d['roofline']['frac'], {k: v.get('value') for k, v in d.get('secondary_workloads', {}).items()})"
exit 0
