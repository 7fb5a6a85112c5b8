#!/bin/bash
# round 6: head.conv1's batched K = 192 Winograd GEMMs on the weight-stationary
# kernel (POSFEAT_WSB=1) vs the 128 x 192 bf6x tile: the A/B test, layer
# timing x2 each
set -e
tag=r16zz3
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
$chk 400 $o/tests.log python -u -m pytest tests/test_gpu_fusions.py::test_head_conv1_gemm_weight_stationary -m gpu -q -rf -s --timeout 300 --timeout-method thread
grep -E "passed|failed|^wsb" $o/tests.log | tail -12
for p in 1 2; do for v in 1 0; do
  env POSFEAT_HIP_LIB=$AB POSFEAT_WSB=$v $chk 200 $o/lt_${v}_$p.log python -u tools/layer_timing.py 32
done; done
for f in $o/lt_*.log; do echo "$f $(grep 'main stream' $f | cut -c1-30) $(grep 'conv:head.conv1' $f)"; done
exit 0
