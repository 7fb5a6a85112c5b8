#!/bin/bash
# One measurement pass on the GPU box: GPU suite, smoke, bench line (with the
# CPU leg), kernel trace + stats of the same bench command, PMC traffic of the
# dominant launch, and the training / correlation lines.  Every GPU step runs
# under its own time limit; a fault/timeout ends the call (tools/gpu_check.sh).
# usage: tools/gpu_round.sh <tag> [quick]
set -e
tag=$1
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 900 $o/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
POSFEAT_HIP_LIB=$PWD/posfeat_amd/libposfeat_hip_ab.so $chk 600 $o/gpu_tests_ab.log python -u -m pytest tests/test_gpu_correlation.py tests/test_gpu_train_tap.py -m gpu -x -q -rs --timeout 300 --timeout-method thread
$chk 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
$chk 400 $o/bench.log python bench.py
grep "^{" $o/bench.log > $o/bench.json || true
[ "$2" = quick ] && exit 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$chk 400 $o/prof.log rocprofv3 --kernel-trace --stats -d $o/prof -o b --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline --no-secondary
for c in FETCH_SIZE WRITE_SIZE; do
  t=$(echo $c | tr A-Z a-z | cut -d_ -f1)
  timeout -s KILL 240 rocprofv3 --pmc $c -d $o/pmc/$t -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline --no-secondary > $o/pmc_$t.log 2>&1 || exit 100
done
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES -d $o/pmc/sq -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline --no-secondary > $o/pmc_sq.log 2>&1 || exit 100
$chk 300 $o/bench_train_kp.json python bench.py --workload train_kp --no-cpu-baseline --steps 10
$chk 300 $o/bench_train_desc.json python bench.py --workload train_desc --no-cpu-baseline --steps 10
$chk 300 $o/bench_corr.json python bench.py --workload corr --no-cpu-baseline --steps 20
exit 0
