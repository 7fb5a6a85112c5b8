#!/bin/bash
# round 6: batched tile loads in the image-moment / composite-weight kernels;
# intrinsic side costs, bench, full GPU suite
set -e
tag=r16k
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
POSFEAT_HIP_LIB=$AB POSFEAT_SIDE=0 $chk 300 $o/prof_serial.log rocprofv3 --kernel-trace --stats -d $PWD/$o/prof -o b --output-format csv -- python3 tools/layer_timing.py 32
python3 tools/rocpd_stats.py $(find $PWD/$o/prof -name "*kernel_trace.csv" | head -1) --top 80 > $o/rocprof_serial.txt
$chk 300 $o/bench.log python bench.py --no-cpu-baseline --no-secondary --steps 40
for abl in 0 7; do
  POSFEAT_HIP_LIB=$AB POSFEAT_SIDE_ABL=$abl $chk 300 $o/bench_side_abl$abl.log python bench.py --no-cpu-baseline --no-secondary --steps 40
done
$chk 1200 $o/gpu_tests.log python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread
grep -E "gfuse|band|ring|imgmom|imgstats" $o/rocprof_serial.txt
for f in bench bench_side_abl0 bench_side_abl7; do echo "$f: $(grep '^{' $o/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
tail -3 $o/gpu_tests.log
exit 0
