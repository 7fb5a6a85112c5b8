#!/bin/bash
# gcombine block order, tile rows fastest (default) vs columns fastest (POSFEAT_GC_ORDER=0): tests, bench A/B, launch times
set -o pipefail
mkdir -p gpurun_out/r15b
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench_config.py tests/test_gpu_model.py tests/test_gpu_repeat.py > gpurun_out/r15b/tests.txt 2>&1 || { tail -20 gpurun_out/r15b/tests.txt; exit 1; }
tail -1 gpurun_out/r15b/tests.txt
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for i in 1 2 3; do
  for arm in row col; do
    if [ $arm = col ]; then E="POSFEAT_GC_ORDER=0"; else E="POSFEAT_GC_ORDER=1"; fi
    env POSFEAT_HIP_LIB=$AB $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > gpurun_out/r15b/bench_${arm}$i.json 2> gpurun_out/r15b/bench_${arm}$i.err || { tail gpurun_out/r15b/bench_${arm}$i.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r15b/bench_${arm}$i.json').read().strip().splitlines()[-1]); h=d['roofline_hbm']; print('$arm$i', d['value'], h['label'], h['avg_launch_ms'], h['frac'])"
  done
done
