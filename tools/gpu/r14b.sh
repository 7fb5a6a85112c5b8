#!/bin/bash
# bf6x memory-instruction placement probe (POSFEAT_BF6X_MEMF) on the tap GEMM / F6-sized GEMM
set -o pipefail
mkdir -p gpurun_out/r14b
export POSFEAT_HIP_LIB=posfeat_amd/libposfeat_hip_ab.so
o=gpurun_out/r14b/probe.txt
for t in 29 31 32; do
  timeout -k 10 120 python -u tools/tapgemm_probe.py $t 20 >> $o 2>&1 || exit 1
done
for m in 2 8; do
  POSFEAT_BF6X_MEMF=$m timeout -k 10 120 python -u tools/tapgemm_probe.py 29 20 >> $o 2>&1 || exit 1
done
cat $o
