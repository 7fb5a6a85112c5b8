#!/bin/bash
# round 6: where the weight-stationary tap GEMM's time goes -- layer timing
# with its stores removed (ABL 1), its A loads removed (2), both (3)
set -e
tag=r16zc
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for v in 0 1 2 3; do
  POSFEAT_HIP_LIB=$AB POSFEAT_TAPWS=1 POSFEAT_TAPWS_ABL=$v $chk 200 $o/lt_$v.log python -u tools/layer_timing.py 32
done
for v in 0 1 2 3; do echo "== abl $v $(grep 'main stream' $o/lt_$v.log | cut -c1-40)"; grep -E "up4tap" $o/lt_$v.log; done
exit 0
