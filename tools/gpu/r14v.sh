#!/bin/bash
# wgrad pixel-split cap A/B (POSFEAT_WGRAD_MAXSPLIT 128 / 256 / 512, A/B build): train_desc + per-label timing, fixture tests at 512
set -o pipefail
mkdir -p gpurun_out/r14v
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for cap in 128 512 256; do
  POSFEAT_HIP_LIB=$AB POSFEAT_WGRAD_MAXSPLIT=$cap timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r14v/td_$cap.txt 2>&1 || { tail gpurun_out/r14v/td_$cap.txt; exit 1; }
  grep '^{"metric' gpurun_out/r14v/td_$cap.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cap', d['value'], d['breakdown_ms'])"
done
POSFEAT_HIP_LIB=$AB POSFEAT_WGRAD_MAXSPLIT=512 timeout -k 10 300 python -u tools/train_layer_timing.py 8 > gpurun_out/r14v/tlt_512.txt 2>&1 || exit 1
grep "wgrad" gpurun_out/r14v/tlt_512.txt | head -20
POSFEAT_HIP_LIB=$AB POSFEAT_WGRAD_MAXSPLIT=512 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bb_train.py tests/test_gpu_train_fullsize.py > gpurun_out/r14v/tests_512.txt 2>&1; tail -3 gpurun_out/r14v/tests_512.txt
