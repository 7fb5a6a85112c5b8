#!/bin/bash
# round 6: closing verification after the batched weight-stationary Winograd
# GEMMs -- GPU suite, smoke, bench (CPU leg + secondary lines),
# kernel trace, PMC passes (traffic of the dominant launches)
set -e
tag=r16zz5
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 1200 $o/gpu_tests.log python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread
tail -3 $o/gpu_tests.log
$chk 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
grep smoke $o/smoke.log
$chk 500 $o/bench.log python bench.py
grep "^{" $o/bench.log > $o/bench.json || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$chk 400 $o/prof.log rocprofv3 --kernel-trace --stats -d $PWD/$o/prof -o b --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline --no-secondary
python3 tools/rocpd_stats.py $(find $PWD/$o/prof -name "*kernel_trace.csv" | head -1) --top 70 > $o/rocprof_extract.txt
for c in FETCH_SIZE WRITE_SIZE; do
  t=$(echo $c | tr A-Z a-z | cut -d_ -f1)
  timeout -s KILL 240 rocprofv3 --pmc $c -d $o/pmc/$t -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline --no-secondary > $o/pmc_$t.log 2>&1 || exit 100
done
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES -d $o/pmc/sq -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline --no-secondary > $o/pmc_sq.log 2>&1 || exit 100
for t in fetch write sq; do f=$(find $o/pmc/$t -name "*counter_collection.csv" | head -1); [ -n "$f" ] && [ "$f" != "$o/pmc/$t/pmc_counter_collection.csv" ] && cp "$f" $o/pmc/$t/pmc_counter_collection.csv; true; done
python3 -c "import json; d=json.loads(open('$o/bench.json').read().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d.get('cpu_baseline',{}).get('value'), {k: (v.get('value'), v.get('roofline',{}).get('frac')) for k, v in d.get('secondary_workloads', {}).items()})"
head -12 $o/rocprof_extract.txt
exit 0
