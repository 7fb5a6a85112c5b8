#!/bin/bash
# round 6: the stem on the weight-stationary kernel (G4 gather, POSFEAT_WSSTEM,
# default on) vs the G4 bf6x tile: the bit-identity test and the model tests,
# layer timing x2 each
set -e
tag=r16zs
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
$chk 600 $o/tests.log python -u -m pytest tests/test_gpu_fusions.py::test_stem_weight_stationary tests/test_gpu_model.py -m gpu -q -rf --timeout 300 --timeout-method thread
tail -2 $o/tests.log
for p in 1 2; do for v in 1 0; do
  env POSFEAT_HIP_LIB=$AB POSFEAT_WSSTEM=$v $chk 200 $o/lt_${v}_$p.log python -u tools/layer_timing.py 32
done; done
for f in $o/lt_*.log; do echo "$f $(grep 'main stream' $f | cut -c1-30) $(grep 'conv:firstconv' $f)"; done
exit 0
