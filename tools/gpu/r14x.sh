#!/bin/bash
# bf6x 128x128 (RB 2) vs 256x128 (RB 4) on the encoder's short-K 1x1 convs
set -o pipefail
mkdir -p gpurun_out/r14x
export PYTHONUNBUFFERED=1 PROBE_SHAPES=enc
for t in 29 31 29 31; do
  timeout -k 10 120 python -u tools/tapgemm_probe.py $t 30 >> gpurun_out/r14x/probe.txt 2>&1 || { tail gpurun_out/r14x/probe.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/r14x/probe.txt
