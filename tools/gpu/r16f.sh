#!/bin/bash
# round 6: intrinsic side-stream kernel costs (serial image branch, A/B build)
# and the kernel trace of the default bench command
set -e
tag=r16f
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
POSFEAT_HIP_LIB=$AB POSFEAT_SIDE=0 $chk 200 $o/lt_serial.log python -u tools/layer_timing.py 32
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$chk 400 $o/prof.log rocprofv3 --kernel-trace --stats -d $PWD/$o/prof -o b --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline --no-secondary
python3 tools/rocpd_stats.py $(find $PWD/$o/prof -name "*kernel_trace.csv" | head -1) --top 70 > $o/rocprof_extract.txt
grep -E "side:|gcombine|head_tail|main stream|gprep|imgstats|gfuse" $o/lt_serial.log
head -12 $o/rocprof_extract.txt
grep -E "gfuse|band|ring|imgmom|imgstats" $o/rocprof_extract.txt
grep "^{" $o/prof.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"])'
exit 0
