#!/bin/bash
# round 6: the head tail with 32-bit indices (POSFEAT_TAIL=46: 74 VGPRs, four
# pairs per step; 47: eight pairs, 126 VGPRs) vs the shipped 43 (90 VGPRs):
# the model tests with 46 and 47, layer timing x2 each
set -e
tag=r16zz
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for v in 46 47; do
  POSFEAT_HIP_LIB=$AB POSFEAT_TAIL=$v $chk 400 $o/tests_$v.log python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_config.py -m gpu -q -rf --timeout 300 --timeout-method thread
  tail -1 $o/tests_$v.log
done
for p in 1 2; do for v in 43 46 47 46b; do
  case $v in 46b) e="POSFEAT_TAIL=46 POSFEAT_TAIL_BLOCKS=16384";; *) e="POSFEAT_TAIL=$v";; esac
  env POSFEAT_HIP_LIB=$AB $e $chk 200 $o/lt_${v}_$p.log python -u tools/layer_timing.py 32
done; done
for f in $o/lt_*.log; do echo "$f $(grep 'main stream' $f | cut -c1-30) $(grep head_tail $f)"; done
exit 0
