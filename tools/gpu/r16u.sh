#!/bin/bash
# round 6: the dense / two-source
# bf6x GEMMs on six-wave 192 x 128 tiles (POSFEAT_BF6X_BM192=1); parity of
# each variant on the model / bench-config tests, the dual-GEMM test, then
# layer timing and bench passes
set -e
tag=r16u
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
$chk 300 $o/dual.log python -u -m pytest tests/test_gpu_ops.py::test_conv1x1_dual_vs_torch -m gpu -q -rf --timeout 120 --timeout-method thread
tail -2 $o/dual.log
POSFEAT_HIP_LIB=$AB POSFEAT_BF6X_BM192=1 $chk 400 $o/tests_bm.log python -u -m pytest tests/test_gpu_ops.py::test_conv1x1_dual_vs_torch tests/test_gpu_model.py tests/test_gpu_bench_config.py -m gpu -q -rf --timeout 300 --timeout-method thread
tail -2 $o/tests_bm.log
for v in base bm; do
  case $v in base) e="";; bm) e="POSFEAT_BF6X_BM192=1";; esac
  env POSFEAT_HIP_LIB=$AB $e $chk 200 $o/lt_$v.log python -u tools/layer_timing.py 32
done
for p in 1 2; do for v in base bm; do
  case $v in base) e="";; bm) e="POSFEAT_BF6X_BM192=1";; esac
  env POSFEAT_HIP_LIB=$AB $e $chk 300 $o/bench_${v}_$p.log python bench.py --no-cpu-baseline --no-secondary --steps 40
done; done
for v in base bm; do echo "== $v $(grep 'main stream' $o/lt_$v.log | cut -c1-40)"; grep "conv:" $o/lt_$v.log | head -24; done
for f in $o/bench_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
exit 0
