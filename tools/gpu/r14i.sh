#!/bin/bash
# F(6x6) input-transform ablations (A/B build, POSFEAT_W6IN_ABL: 1 no V stores, 2 no input loads, 3 neither) in the B=32 layer timing
set -o pipefail
mkdir -p gpurun_out/r14i
export PYTHONUNBUFFERED=1 POSFEAT_HIP_LIB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for a in 0 1 2 3; do
  POSFEAT_W6IN_ABL=$a timeout -k 10 300 python -u tools/layer_timing.py 32 > gpurun_out/r14i/lt_$a.txt 2>&1 || { tail gpurun_out/r14i/lt_$a.txt; exit 1; }
  echo "abl $a"; grep "wino:in:" gpurun_out/r14i/lt_$a.txt | head -5
done
