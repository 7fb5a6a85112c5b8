#!/bin/bash
# round 6: the fused-upsample F(6x6) input transform with its six half-res
# rows loaded first (UPM = 1) vs the two-row window (POSFEAT_W6IN_UPM=0):
# the bit-identity tests, layer timing x2 each
set -e
tag=r16zq
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
$chk 600 $o/tests.log python -u -m pytest tests/test_gpu_bf6r.py tests/test_gpu_model.py -m gpu -q -rf --timeout 300 --timeout-method thread
tail -2 $o/tests.log
for p in 1 2; do for v in 1 0; do
  env POSFEAT_HIP_LIB=$AB POSFEAT_W6IN_UPM=$v $chk 200 $o/lt_${v}_$p.log python -u tools/layer_timing.py 32
done; done
for f in $o/lt_*.log; do echo "$f $(grep 'main stream' $f | cut -c1-30)"; grep -E "wino:in:upconv" $f; done
exit 0
