#!/bin/bash
# probe: A loads as whole 128-B lines (8 rows per instruction, wrong operand layout: timing only) vs the shipped 16 rows x 64 B
set -o pipefail
mkdir -p gpurun_out/r15a
export PYTHONUNBUFFERED=1 POSFEAT_HIP_LIB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for i in 1 2; do
  timeout -k 10 120 python -u tools/tapgemm_probe.py 29 20 >> gpurun_out/r15a/probe.txt 2>&1 || exit 1
  POSFEAT_BF6X_AL=1 timeout -k 10 120 python -u tools/tapgemm_probe.py 29 20 2>&1 | sed 's/^/AL /' >> gpurun_out/r15a/probe.txt || exit 1
done
grep -v amdgpu.ids gpurun_out/r15a/probe.txt
