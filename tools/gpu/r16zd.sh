#!/bin/bash
# round 6: weight-stationary tap GEMM variants -- prefetch distance 2 (PD) and
# twelve waves (three per SIMD, NW) -- parity (bit-identity test) of each,
# layer timing of each, bench of the default and the variants
set -e
tag=r16zd
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for v in pd2 nw12; do
  case $v in pd2) e="POSFEAT_TAPWS_PD=2";; nw12) e="POSFEAT_TAPWS_NW=12";; esac
  env $e $chk 300 $o/tests_$v.log python -u -m pytest tests/test_gpu_fusions.py::test_tap_gemm_weight_stationary -m gpu -q -rf -s --timeout 300 --timeout-method thread
  grep -E "passed|failed|tapws" $o/tests_$v.log | tail -3
done
for v in base ws pd2 nw12; do
  case $v in base) e="";; ws) e="POSFEAT_TAPWS=1";; pd2) e="POSFEAT_TAPWS=1 POSFEAT_TAPWS_PD=2";; nw12) e="POSFEAT_TAPWS=1 POSFEAT_TAPWS_NW=12";; esac
  env POSFEAT_HIP_LIB=$AB $e $chk 200 $o/lt_$v.log python -u tools/layer_timing.py 32
done
for p in 1 2; do for v in ws pd2 nw12; do
  case $v in ws) e="POSFEAT_TAPWS=1";; pd2) e="POSFEAT_TAPWS=1 POSFEAT_TAPWS_PD=2";; nw12) e="POSFEAT_TAPWS=1 POSFEAT_TAPWS_NW=12";; esac
  env POSFEAT_HIP_LIB=$AB $e $chk 300 $o/bench_${v}_$p.log python bench.py --no-cpu-baseline --no-secondary --steps 40
done; done
for v in base ws pd2 nw12; do echo "== $v $(grep 'main stream' $o/lt_$v.log | cut -c1-40)"; grep -E "up4tap" $o/lt_$v.log; done
for f in $o/bench_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')"; done
exit 0
