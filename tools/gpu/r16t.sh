#!/bin/bash
# round 6: head.conv2's tap GEMM + combine in image chunks through one P slab
# (A/B POSFEAT_HEAD_CHUNK=G) -- parity with chunks, then layer timing and
# bench at G = 0 (whole batch), 1, 2, 4 on one box; also the dual-GEMM test
set -e
tag=r16t
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
$chk 300 $o/dual.log python -u -m pytest tests/test_gpu_ops.py::test_conv1x1_dual_vs_torch -m gpu -q -rf --timeout 120 --timeout-method thread
tail -2 $o/dual.log
POSFEAT_HIP_LIB=$AB POSFEAT_HEAD_CHUNK=2 $chk 400 $o/tests_c2.log python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_config.py -m gpu -q -rf --timeout 300 --timeout-method thread
tail -2 $o/tests_c2.log
for g in 0 1 2 4; do
  POSFEAT_HIP_LIB=$AB POSFEAT_HEAD_CHUNK=$g $chk 200 $o/lt_$g.log python -u tools/layer_timing.py 32
done
for p in 1 2; do for g in 0 2 1; do
  POSFEAT_HIP_LIB=$AB POSFEAT_HEAD_CHUNK=$g $chk 300 $o/bench_${g}_$p.log python bench.py --no-cpu-baseline --no-secondary --steps 40
done; done
for g in 0 1 2 4; do echo "== $g $(grep 'main stream' $o/lt_$g.log | cut -c1-40)"; grep -E "up4tap|gcombine" $o/lt_$g.log; done
for f in $o/bench_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
exit 0
