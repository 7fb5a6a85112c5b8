#!/bin/bash
# Counter passes over the head.conv2-shaped probe (tools/conv2_probe.py).
# One rocprofv3 run per counter group (SQ/GRBM, TCC FETCH, TCC WRITE, LDS).
# usage: [PROBE=tools/up4_probe.py] tools/pmc_conv2.sh <outdir>
out=${1:-gpurun_out/pmc}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
run() {
  tag=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" -d "$out/$tag" -o pmc --output-format csv \
    -- python3 ${PROBE:-tools/conv2_probe.py} 8 3 > "$out/$tag.log" 2>&1
  rc=$?
  echo "[pmc] $tag rc=$rc" >> "$out/$tag.log"
  [ $rc -lt 124 ] || exit 100
}
run sq GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS
run fetch FETCH_SIZE
run write WRITE_SIZE
