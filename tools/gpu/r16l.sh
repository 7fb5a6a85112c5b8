#!/bin/bash
# round 6: where the image branch forks (POSFEAT_SIDE_AT, A/B build), two passes
set -e
tag=r16l
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for pass in 1 2; do
  for at in 2 3 4 1; do
    POSFEAT_HIP_LIB=$AB POSFEAT_SIDE_AT=$at $chk 300 $o/bench_at${at}_p$pass.log python bench.py --no-cpu-baseline --no-secondary --steps 40
  done
done
for f in $o/bench_at*.log; do echo "$f: $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
exit 0
