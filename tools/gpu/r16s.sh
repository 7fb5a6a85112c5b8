#!/bin/bash
# round 6: conv3 + downsample as one two-source GEMM (pf_conv_dual) -- model /
# extraction tests, layer timing and bench with the fusion (default) and without
# (A/B library, POSFEAT_DSFUSE=0), two passes each
set -e
tag=r16s
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
$chk 600 $o/tests.log python -u -m pytest tests/test_gpu_ops.py::test_conv1x1_dual_vs_torch tests/test_gpu_model.py tests/test_gpu_api.py tests/test_gpu_bench_config.py tests/test_gpu_extract.py tests/test_gpu_precision.py -m gpu -q -rf --timeout 300 --timeout-method thread
tail -3 $o/tests.log
$chk 200 $o/lt_new.log python -u tools/layer_timing.py 32
POSFEAT_HIP_LIB=$AB POSFEAT_DSFUSE=0 $chk 200 $o/lt_old.log python -u tools/layer_timing.py 32
for p in 1 2; do
  $chk 300 $o/bench_new_$p.log python bench.py --no-cpu-baseline --no-secondary --steps 40
  POSFEAT_HIP_LIB=$AB POSFEAT_DSFUSE=0 $chk 300 $o/bench_old_$p.log python bench.py --no-cpu-baseline --no-secondary --steps 40
done
for v in new old; do echo "== $v $(grep 'main stream' $o/lt_$v.log | cut -c1-40)"; grep -E "layer[123]\.0\.(conv3|downsample)" $o/lt_$v.log; done
for f in $o/bench_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
exit 0
