#!/bin/bash
# round 6: the autotune choices (candidates and times) of the encoder's 1x1
# convs, layer3.0.conv1 (0.43 ms at 93 TF/s) against layer2.x.conv1 (165)
set -e
tag=r16zp
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
POSFEAT_TILE_DB=0 POSFEAT_AUTOTUNE_LOG=1 $chk 200 $o/lt.log python -u tools/layer_timing.py 32
grep -E "autotune\] (layer3.0|layer2.1|layer2.0)" $o/lt.log || true
grep -E "conv:layer3.0|conv:layer2.1.conv1" $o/lt.log
exit 0
