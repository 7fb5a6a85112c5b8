#!/bin/bash
# round 6: head tail, waves interleaved over the pixels (A/B POSFEAT_TAIL=42
# nontemporal / 43 plain) vs contiguous ranges (41), x2; blocks 16384 at 42
set -e
tag=r16zm
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for p in 1 2; do for v in 41 42 43 42b; do
  case $v in 42b) e="POSFEAT_TAIL=42 POSFEAT_TAIL_BLOCKS=2048";; *) e="POSFEAT_TAIL=$v";; esac
  env POSFEAT_HIP_LIB=$AB $e $chk 200 $o/lt_${v}_$p.log python -u tools/layer_timing.py 32
done; done
for f in $o/lt_*.log; do echo "$f $(grep 'main stream' $f | cut -c1-30) $(grep head_tail $f)"; done
exit 0
