#!/bin/bash
# round 6: head_tail_conv3_kernel without a 64-bit division per pixel: the
# model / bench-config tests, layer timing x3
set -e
tag=r16zl
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 600 $o/tests.log python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_config.py -m gpu -q -rf --timeout 300 --timeout-method thread
tail -2 $o/tests.log
for p in 1 2 3; do
  $chk 200 $o/lt_$p.log python -u tools/layer_timing.py 32
done
for p in 1 2 3; do echo "== $p $(grep 'main stream' $o/lt_$p.log | cut -c1-40)"; grep -E "head_tail|up4tap" $o/lt_$p.log; done
exit 0
