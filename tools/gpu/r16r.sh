#!/bin/bash
# round 6: rank on 64-bit composite keys (one compare per entry) -- detection
# tests, kernel trace, one e2e run for the construction phases
set -e
tag=r16r
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
$chk 600 $o/tests.log python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_api.py tests/test_gpu_bench_config.py tests/test_gpu_extract.py -m gpu -q -rf --timeout 300 --timeout-method thread
tail -3 $o/tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$chk 300 $o/prof_new.log rocprofv3 --kernel-trace --stats -d $PWD/$o/prof_new -o b --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline --no-secondary
for v in new; do
  python3 tools/rocpd_stats.py $(find $PWD/$o/prof_$v -name "*kernel_trace.csv" | head -1) --top 70 > $o/rocprof_$v.txt
  echo "== $v $(grep '^{' $o/prof_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  grep -E "det_|total" $o/rocprof_$v.txt
done
$chk 400 $o/e2e_480.log python -u tools/extract_e2e.py --seqs 96 --sizes 480x640 --passes 1
grep -o '"setup[^}]*}' $o/e2e_480.log || true
exit 0
