#!/bin/bash
# round 6: the tap GEMM instance without the conv epilogue (EP = 0, 158 VGPRs
# as before the generalisation): fusion tests, layer timing x2
set -e
tag=r16zk
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 600 $o/tests.log python -u -m pytest tests/test_gpu_fusions.py -m gpu -q -rf --timeout 300 --timeout-method thread
tail -2 $o/tests.log
for p in 1 2 3; do
  $chk 200 $o/lt_$p.log python -u tools/layer_timing.py 32
done
for p in 1 2 3; do echo "== $p $(grep 'main stream' $o/lt_$p.log | cut -c1-40)"; grep -E "gcombine|up4tap|layer1.[12].conv1 " $o/lt_$p.log; done
exit 0
