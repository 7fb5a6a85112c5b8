#!/bin/bash
# round 6: the short-K dense 1x1 convs on the weight-stationary kernel
# (POSFEAT_WS1X1, default on) vs the tuned bf6x tiles (POSFEAT_WS1X1=0):
# the A/B fusion tests, then per-layer timing both ways
set -e
tag=r16zh
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
$chk 600 $o/tests.log python -u -m pytest tests/test_gpu_fusions.py tests/test_gpu_ops.py -m gpu -q -rf -s --timeout 300 --timeout-method thread
grep -E "passed|failed|ws1x1" $o/tests.log | tail -14
for p in 1 2; do for v in ws tiles; do
  case $v in ws) e="";; tiles) e="POSFEAT_WS1X1=0";; esac
  env POSFEAT_HIP_LIB=$AB $e $chk 200 $o/lt_${v}_$p.log python -u tools/layer_timing.py 32
done; done
for f in $o/lt_*.log; do echo "== $f $(grep 'main stream' $f | cut -c1-40)"; grep -E "conv:layer[123]\.[0-9]\.conv[13] |conv:conv_fine|conv:layer2.0.conv1" $f | head -30; done
exit 0
