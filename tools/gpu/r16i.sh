#!/bin/bash
# round 6: head tail kernel A/B (pairs in flight, nontemporal loads, grid)
set -e
tag=r16i
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for v in 40 41 80 81; do
  POSFEAT_HIP_LIB=$AB POSFEAT_TAIL=$v $chk 200 $o/lt_tail$v.log python -u tools/layer_timing.py 32
done
for nb in 4096 16384 32768; do
  POSFEAT_HIP_LIB=$AB POSFEAT_TAIL_BLOCKS=$nb $chk 200 $o/lt_tailb$nb.log python -u tools/layer_timing.py 32
done
for f in $o/lt_tail*.log; do echo "$f $(grep -E 'head_tail' $f)"; done
exit 0
