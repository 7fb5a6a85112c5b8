#!/bin/bash
# bf6x: weights as the MFMA A operand, results stored straight from the registers: probe, tests, bench A/B against f9475ea
set -o pipefail
mkdir -p gpurun_out/r14g
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
REF=$PWD/abref/libposfeat_hip_f9475ea.so
o=gpurun_out/r14g/probe.txt
for t in 29 31 32; do
  timeout -k 10 120 python -u tools/tapgemm_probe.py $t 20 >> $o 2>&1 || { tail $o; exit 1; }
  POSFEAT_HIP_LIB=$REF timeout -k 10 120 python -u tools/tapgemm_probe.py $t 20 2>&1 | sed 's/^/ref /' >> $o || exit 1
done
grep -v amdgpu.ids $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bf6x.py tests/test_gpu_tiles.py tests/test_gpu_bench_config.py tests/test_gpu_bf6r.py \
  tests/test_gpu_model.py tests/test_gpu_ops.py > gpurun_out/r14g/tests.txt 2>&1 || { tail -30 gpurun_out/r14g/tests.txt; exit 1; }
tail -2 gpurun_out/r14g/tests.txt
for i in 1 2; do
  for arm in new ref; do
    if [ $arm = ref ]; then L=$REF; else L=$PWD/posfeat_amd/libposfeat_hip.so; fi
    POSFEAT_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r14g/bench_${arm}$i.json 2> gpurun_out/r14g/bench_${arm}$i.err || { tail gpurun_out/r14g/bench_${arm}$i.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r14g/bench_${arm}$i.json').read().strip().splitlines()[-1]); print('$arm$i', d['value'], d['roofline']['frac'], d['roofline'].get('avg_launch_ms'))"
  done
done
