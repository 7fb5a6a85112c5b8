#!/bin/bash
# Wave-state and instruction-mix counter passes over a short bench.py run
# (one rocprofv3 --pmc run per group), summarised per kernel by
# tools/pmc_summary.py.  usage: [BENCH_ARGS="--workload corr ..."] tools/pmc_kernels.sh <outdir>
out=${1:-gpurun_out/pmck}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
run() {
  tag=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" -d "$out/$tag" -o pmc --output-format csv \
    -- python3 bench.py ${BENCH_ARGS:---steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline --no-secondary} \
    > "$out/$tag.log" 2>&1
  rc=$?
  echo "[pmc] $tag rc=$rc" >> "$out/$tag.log"
  [ $rc -lt 124 ] || exit 100
}
run sq GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU
exit 0
