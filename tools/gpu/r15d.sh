#!/bin/bash
# F(6x6) transforms with an XCD-aware block order (default) vs round-robin (POSFEAT_WINO_XCD=0): tests, layer timing, bench A/B
set -o pipefail
mkdir -p gpurun_out/r15d
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_bf6r.py tests/test_gpu_bench_config.py tests/test_bb_train.py > gpurun_out/r15d/tests.txt 2>&1 || { tail -20 gpurun_out/r15d/tests.txt; exit 1; }
tail -1 gpurun_out/r15d/tests.txt
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for arm in 1 0; do
  env POSFEAT_HIP_LIB=$AB POSFEAT_WINO_XCD=$arm timeout -k 10 300 python -u tools/layer_timing.py 32 > gpurun_out/r15d/lt_$arm.txt 2>&1 || exit 1
  echo "xcd $arm: $(grep 'wino:' gpurun_out/r15d/lt_$arm.txt | awk '{s+=$3} END {print s}') ms of transforms"
done
for i in 1 2 3; do
  for arm in 1 0; do
    env POSFEAT_HIP_LIB=$AB POSFEAT_WINO_XCD=$arm timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > gpurun_out/r15d/bench_${arm}_$i.json 2> gpurun_out/r15d/bench_${arm}_$i.err || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/r15d/bench_${arm}_$i.json').read().strip().splitlines()[-1]); print('xcd $arm/$i', d['value'])"
  done
done
