#!/bin/bash
# gcombine block order: rows fastest (1) vs strips of 2 / 4 tile columns (A/B build), bench + gcombine launch time
set -o pipefail
mkdir -p gpurun_out/r15c
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
timeout -k 10 600 env POSFEAT_HIP_LIB=$AB POSFEAT_GC_ORDER=2 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench_config.py > gpurun_out/r15c/tests2.txt 2>&1 || { tail -20 gpurun_out/r15c/tests2.txt; exit 1; }
tail -1 gpurun_out/r15c/tests2.txt
for i in 1 2; do
  for o in 1 2 4; do
    env POSFEAT_HIP_LIB=$AB POSFEAT_GC_ORDER=$o timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > gpurun_out/r15c/bench_${o}_$i.json 2> gpurun_out/r15c/bench_${o}_$i.err || { tail gpurun_out/r15c/bench_${o}_$i.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r15c/bench_${o}_$i.json').read().strip().splitlines()[-1]); h=d['roofline_hbm']; print('order $o/$i', d['value'], h['avg_launch_ms'], h['frac'])"
  done
done
