#!/bin/bash
# bf6x ablations on the tap GEMM / F6-sized GEMM: 17 no loop loads, 33 no MFMAs, 65 no epilogue, 81 neither loads nor epilogue
set -o pipefail
mkdir -p gpurun_out/r14c
export POSFEAT_HIP_LIB=posfeat_amd/libposfeat_hip_ab.so
o=gpurun_out/r14c/probe.txt
for m in 1 17 33 65 81; do
  POSFEAT_BF6X_MEMF=$m timeout -k 10 120 python -u tools/tapgemm_probe.py 29 20 >> $o 2>&1 || exit 1
done
grep -v amdgpu.ids $o
