#!/bin/bash
# extraction bench A/B: HEAD (bf6x tiles without the BN epilogue mode) against the session-start library (d21ea03)
set -o pipefail
mkdir -p gpurun_out/r14q
export PYTHONUNBUFFERED=1
REF=$PWD/abref/libposfeat_hip_d21ea03.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bf6x.py tests/test_gpu_tiles.py tests/test_gpu_bench_config.py tests/test_bb_train.py > gpurun_out/r14q/tests.txt 2>&1 || { tail -20 gpurun_out/r14q/tests.txt; exit 1; }
tail -1 gpurun_out/r14q/tests.txt
for i in 1 2 3; do
  for arm in new ref; do
    if [ $arm = ref ]; then L=$REF; else L=$PWD/posfeat_amd/libposfeat_hip.so; fi
    POSFEAT_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > gpurun_out/r14q/bench_${arm}$i.json 2> gpurun_out/r14q/bench_${arm}$i.err || { tail gpurun_out/r14q/bench_${arm}$i.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r14q/bench_${arm}$i.json').read().strip().splitlines()[-1]); print('$arm$i', d['value'], d['roofline']['frac'])"
  done
done
