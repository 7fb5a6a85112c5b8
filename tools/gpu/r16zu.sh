#!/bin/bash
# round 6: the fused-upsample transform forced to four waves per SIMD
# (POSFEAT_W6IN_WPE=4: 128 VGPRs, 24 spilled) vs three (138 VGPRs), x2
set -e
tag=r16zu
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for p in 1 2; do for v in 4 1; do
  env POSFEAT_HIP_LIB=$AB POSFEAT_W6IN_WPE=$v $chk 200 $o/lt_${v}_$p.log python -u tools/layer_timing.py 32
done; done
for f in $o/lt_*.log; do echo "$f $(grep 'main stream' $f | cut -c1-30)"; grep -E "wino:in:upconv" $f; done
exit 0
