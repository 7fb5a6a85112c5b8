#!/bin/bash
# round 6: F(6x6) transforms one channel per thread (fewer VGPRs, more waves), A/B
set -e
tag=r16m
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for v in 00 11 00 11 10 01; do
  POSFEAT_HIP_LIB=$AB POSFEAT_W6IN_VW1=${v:0:1} POSFEAT_W6OUT_VW1=${v:1:1} $chk 200 $o/lt_$v.log python -u tools/layer_timing.py 32
  cp $o/lt_$v.log $o/lt_${v}_$(date +%s%N).log
done
for v in 00 11; do
  POSFEAT_HIP_LIB=$AB POSFEAT_W6IN_VW1=${v:0:1} POSFEAT_W6OUT_VW1=${v:1:1} $chk 300 $o/bench_$v.log python bench.py --no-cpu-baseline --no-secondary --steps 40
done
for f in $o/lt_??_*.log; do echo "$f $(grep 'main stream' $f | cut -c1-30)"; grep -E "wino:(in|out):(upconv|iconv|head)" $f; done
for v in 00 11; do echo "bench $v: $(grep '^{' $o/bench_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
exit 0
