#!/bin/bash
# head.conv2 in two batch halves over the main and side streams: tests, bench A/B (POSFEAT_HEAD2S=0), layer timing
set -o pipefail
mkdir -p gpurun_out/r14k
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bench_config.py tests/test_gpu_model.py tests/test_gpu_repeat.py tests/test_gpu_api.py \
  > gpurun_out/r14k/tests.txt 2>&1 || { tail -30 gpurun_out/r14k/tests.txt; exit 1; }
tail -2 gpurun_out/r14k/tests.txt
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for i in 1 2; do
  for arm in on off; do
    if [ $arm = off ]; then E="POSFEAT_HEAD2S=0"; else E="POSFEAT_HEAD2S=1"; fi
    env POSFEAT_HIP_LIB=$AB $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > gpurun_out/r14k/bench_${arm}$i.json 2> gpurun_out/r14k/bench_${arm}$i.err || { tail gpurun_out/r14k/bench_${arm}$i.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r14k/bench_${arm}$i.json').read().strip().splitlines()[-1]); r=d['roofline']; h=d.get('roofline_hbm',{}); print('$arm$i', d['value'], r['kernel'][:40], r['frac'], r.get('avg_launch_ms'), h.get('label'), h.get('avg_launch_ms'), h.get('frac'))"
  done
done
timeout -k 10 300 python -u tools/layer_timing.py 32 > gpurun_out/r14k/lt_on.txt 2>&1 || exit 1
head -16 gpurun_out/r14k/lt_on.txt
