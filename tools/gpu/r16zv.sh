#!/bin/bash
# round 6: the head tail walking the pixels last-first (POSFEAT_TAIL=44: the
# most recently written y may still be in the memory-side cache) vs first-last
# (43, the default), x2; the tail's parity tests with 44
set -e
tag=r16zv
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
POSFEAT_HIP_LIB=$AB POSFEAT_TAIL=44 $chk 400 $o/tests.log python -u -m pytest tests/test_gpu_model.py -m gpu -q -rf --timeout 300 --timeout-method thread
tail -2 $o/tests.log
for p in 1 2; do for v in 44 43; do
  env POSFEAT_HIP_LIB=$AB POSFEAT_TAIL=$v $chk 200 $o/lt_${v}_$p.log python -u tools/layer_timing.py 32
done; done
for f in $o/lt_*.log; do echo "$f $(grep 'main stream' $f | cut -c1-30) $(grep head_tail $f)"; done
exit 0
