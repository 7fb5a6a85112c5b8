#!/bin/bash
# round 6: XCD-aware block order of the weight-stationary tap GEMM (the nine
# column-tile blocks of an M-tile walk on one XCD) vs the plain order
# (POSFEAT_TAPWS_ABL=4); bit-identity test; the failing bf6r test re-run
set -e
tag=r16zg
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
$chk 600 $o/tests.log python -u -m pytest tests/test_gpu_fusions.py tests/test_gpu_bf6r.py -m gpu -q -rf --timeout 300 --timeout-method thread
tail -2 $o/tests.log
for p in 1 2; do for v in xcd plain; do
  case $v in xcd) e="";; plain) e="POSFEAT_TAPWS_ABL=4";; esac
  env POSFEAT_HIP_LIB=$AB $e $chk 200 $o/lt_${v}_$p.log python -u tools/layer_timing.py 32
done; done
for f in $o/lt_*.log; do echo "== $f $(grep 'main stream' $f | cut -c1-40)"; grep -E "up4tap" $f; done
exit 0
