#!/bin/bash
# round 6: head.conv2's tap GEMM on the weight-stationary persistent kernel
# (POSFEAT_TAPWS=1) -- its fusion test, layer timing and bench with / without
set -e
tag=r16zb
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
$chk 600 $o/tests.log python -u -m pytest tests/test_gpu_fusions.py::test_tap_gemm_weight_stationary -m gpu -q -rf -s --timeout 300 --timeout-method thread
grep -E "passed|failed|tapws" $o/tests.log | tail -8
for v in base ws; do
  case $v in base) e="";; ws) e="POSFEAT_TAPWS=1";; esac
  env POSFEAT_HIP_LIB=$AB $e $chk 200 $o/lt_$v.log python -u tools/layer_timing.py 32
done
for p in 1 2; do for v in base ws; do
  case $v in base) e="";; ws) e="POSFEAT_TAPWS=1";; esac
  env POSFEAT_HIP_LIB=$AB $e $chk 300 $o/bench_${v}_$p.log python bench.py --no-cpu-baseline --no-secondary --steps 40
done; done
for v in base ws; do echo "== $v $(grep 'main stream' $o/lt_$v.log | cut -c1-40)"; grep -E "up4tap|gcombine" $o/lt_$v.log; done
for f in $o/bench_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')"; done
exit 0
