#!/bin/bash
# One iteration on the GPU box: selected GPU tests, the bench line, and a
# kernel trace of the same bench command summarised per (kernel, grid).
# Every GPU step runs under its own time limit; a fault or timeout ends the
# call (tools/gpu_check.sh).
# usage: tools/gpu_iter.sh <tag> "<pytest targets>" [bench args...]
#   an empty test string skips the tests; "none" skips the trace as well
set -e
tag=$1; tests=$2; shift 2
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
if [ -n "$tests" ] && [ "$tests" != none ]; then
  $chk 600 $o/gpu_tests.log python -u -m pytest $tests -m gpu -x -q --timeout 240 --timeout-method thread
  grep -E "passed|failed|error" $o/gpu_tests.log | tail -2 || true
fi
$chk 300 $o/bench.log python bench.py "$@"
grep "^{" $o/bench.log > $o/bench.json || true
[ "$tests" = none ] && exit 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$chk 300 $o/prof.log rocprofv3 --kernel-trace --stats -d $o/prof -o b --output-format csv -- python3 bench.py --steps 10 --no-cpu-baseline "$@"
f=$(ls $o/prof/*/b_kernel_trace.csv $o/prof/b_kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && python tools/prof_summary.py "$f" 40 > $o/kernels.txt
exit 0
