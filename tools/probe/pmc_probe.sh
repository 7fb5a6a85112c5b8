#!/bin/bash
# SQ counter passes over the GEMM probe (one rocprofv3 run per counter group).
# usage: tools/probe/pmc_probe.sh <outdir>
out=${1:-gpurun_out/pmcp}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
run() {
  tag=$1; shift
  timeout -s KILL 60 rocprofv3 --pmc "$@" -d "$out/$tag" -o pmc --output-format csv \
    -- probe_build/gemm_probe 3 > "$out/$tag.log" 2>&1
  rc=$?
  echo "[pmc] $tag rc=$rc" >> "$out/$tag.log"
  [ $rc -lt 124 ] || exit 100
}
run sq GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU
exit 0
