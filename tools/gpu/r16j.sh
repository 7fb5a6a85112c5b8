#!/bin/bash
# round 6: the 128x256 bf16x6 tile for the decoder's batched Winograd GEMMs (A/B)
set -e
tag=r16j
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for v in 0 1 0 1; do
  POSFEAT_HIP_LIB=$AB POSFEAT_BF6X_N256=$v $chk 200 $o/lt_n256_$v.log python -u tools/layer_timing.py 32
  cp $o/lt_n256_$v.log $o/lt_n256_${v}_$(date +%s%N).log
done
for f in $o/lt_n256_*_*.log; do echo "$f"; grep -E "main stream|wino:? ?|conv:(up|i)conv" $f | grep -E "main stream|conv:" ; done
exit 0
