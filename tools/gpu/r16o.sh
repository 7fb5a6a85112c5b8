#!/bin/bash
# round 6: keypoint-head training -- the adjoint combine at 2 low-res rows per block (A/B)
set -e
tag=r16o
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for v in 4 2 4 2; do
  POSFEAT_HIP_LIB=$AB POSFEAT_ADJ_TQ=$v $chk 300 $o/kp_tq$v.log python bench.py --workload train_kp --steps 10 --warmup 3 --no-cpu-baseline
  cp $o/kp_tq$v.log $o/kp_tq${v}_$(date +%s%N).log
done
for f in $o/kp_tq?_*.log; do echo "$f: $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["breakdown_ms"]["top_labels"].get("bwd:up4tap_adjoint"), d["breakdown_ms"]["top_labels"].get("bwd:tail"))')"; done
exit 0
