#!/bin/bash
# round 6: layer timing on the final tree (the weight-stationary paths active)
set -e
tag=r16zz8
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 200 $o/lt.log python -u tools/layer_timing.py 32
grep -E "main stream|conv:head.conv1.wino|conv:layer2.1.conv2.wino|conv:layer3.1.conv2.wino|up4tap|layer1.1.conv1 |head_tail|wino:in:upconv2" $o/lt.log
exit 0
