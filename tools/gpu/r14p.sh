#!/bin/bash
# extraction bench A/B: HEAD against the session-start library (d21ea03), interleaved pairs, same box
set -o pipefail
mkdir -p gpurun_out/r14p
export PYTHONUNBUFFERED=1
REF=$PWD/abref/libposfeat_hip_d21ea03.so
for i in 1 2 3; do
  for arm in new ref; do
    if [ $arm = ref ]; then L=$REF; else L=$PWD/posfeat_amd/libposfeat_hip.so; fi
    POSFEAT_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > gpurun_out/r14p/bench_${arm}$i.json 2> gpurun_out/r14p/bench_${arm}$i.err || { tail gpurun_out/r14p/bench_${arm}$i.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r14p/bench_${arm}$i.json').read().strip().splitlines()[-1]); print('$arm$i', d['value'], d['roofline']['frac'])"
  done
done
