#!/bin/bash
# round 6: run-to-run range of the headline bench on one box (three runs of
# the default bench.py extract line without the CPU leg / secondary lines)
set -e
tag=r16zy
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
for p in 1 2 3; do
  $chk 300 $o/bench_$p.log python bench.py --no-cpu-baseline --no-secondary
done
for p in 1 2 3; do grep "^{" $o/bench_$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"; done
exit 0
