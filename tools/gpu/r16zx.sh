#!/bin/bash
# round 6: kernel trace of the correlation workload (bench.py --workload corr)
set -e
tag=r16zx
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$chk 300 $o/prof.log rocprofv3 --kernel-trace --stats -d $PWD/$o/prof -o c --output-format csv -- python3 bench.py --workload corr --steps 20 --no-cpu-baseline
python3 tools/rocpd_stats.py $(find $PWD/$o/prof -name "*kernel_trace.csv" | head -1) --top 30 > $o/rocprof_corr.txt
rm -rf $o/prof
head -32 $o/rocprof_corr.txt
grep "^{" $o/prof.log | cut -c1-300 || true
exit 0
