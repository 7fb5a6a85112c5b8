#!/bin/bash
# round 6: batched weight-stationary GEMMs -- POSFEAT_WSB 1 (default: head.conv1
# K = 192), 0 (bf6x tiles), 2 (+ layer2 conv2 K = 128), 3 (+ layer3 conv2
# K = 256): the A/B tests (0 and 3 vs the default), the train_kp tests, layer
# timing x2 each
set -e
tag=r16zz4
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
$chk 600 $o/tests.log python -u -m pytest tests/test_gpu_fusions.py::test_head_conv1_gemm_weight_stationary tests/test_gpu_train_tap.py tests/test_gpu_model.py -m gpu -q -rf -s --timeout 300 --timeout-method thread
grep -E "passed|failed|^wsb" $o/tests.log | grep -v "True$" | tail -8
for p in 1 2; do for v in 1 0 2 3; do
  env POSFEAT_HIP_LIB=$AB POSFEAT_WSB=$v $chk 200 $o/lt_${v}_$p.log python -u tools/layer_timing.py 32
done; done
for f in $o/lt_*.log; do echo "$f $(grep 'main stream' $f | cut -c1-30)"; grep -E "conv:head.conv1.wino|conv:layer2.1.conv2.wino|conv:layer3.1.conv2.wino" $f; done
exit 0
