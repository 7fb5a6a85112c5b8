#!/bin/bash
# Same-box A/B of bench.py under environment settings, interleaved pairs,
# plus per-layer timing for each arm.
# usage: tools/ab_run.sh <tag> <pairs> "<envA>" "<envB>" [extra bench args]
tag=$1; pairs=$2; A=$3; B=$4; shift 4
o=gpurun_out/$tag; mkdir -p $o
for i in $(seq 1 $pairs); do
  for arm in A B; do
    [ $arm = A ] && e=$A || e=$B
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $o/bench_${arm}$i.json 2> $o/bench_${arm}$i.err || exit 100
    grep -o '"value": [0-9.]*' $o/bench_${arm}$i.json | head -1 | sed "s#^#$arm$i ($e) #"
  done
done
for arm in A B; do
  [ $arm = A ] && e=$A || e=$B
  env $e timeout -k 10 300 python tools/layer_timing.py 32 > $o/lt_$arm.txt 2>&1 || exit 100
done
exit 0
