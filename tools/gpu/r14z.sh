#!/bin/bash
# memory-path counters of the extraction step (separate --pmc passes, no tracing domains): TA/TD busy, TA stalls on TCP, L1->L2 latency, L2 hits
o=gpurun_out/r14z
mkdir -p $o
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
run() {
  tag=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" -d $PWD/$o/$tag -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline --no-secondary > $o/$tag.log 2>&1
  rc=$?
  echo "[pmc] $tag rc=$rc"
  [ $rc -lt 124 ] || exit 100
}
run ta GRBM_GUI_ACTIVE TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum || exit 1
run td GRBM_GUI_ACTIVE TD_TD_BUSY_sum || exit 1
run tcc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum || exit 1
run tcp GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum || exit 1
python3 tools/pmc_mem.py $(find $PWD/$o -name "*counter_collection.csv") > $o/pmc_mem.txt 2>&1
cat $o/pmc_mem.txt
find $o -name "*.csv" -size +20M -delete
