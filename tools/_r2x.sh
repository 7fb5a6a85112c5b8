set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
POSFEAT_BF6=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d gpurun_out/pmc_r2x -o pmc --output-format csv -- python tools/layer_timing.py 8 480 640 > gpurun_out/pmc_r2x.log 2>&1
