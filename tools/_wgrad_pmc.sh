set -e
mkdir -p gpurun_out/pmc_wg
timeout -k 10 120 python tools/wgrad_probe.py 8 5 > gpurun_out/pmc_wg/time.log 2>&1
timeout -k 10 120 python tools/wgrad_probe.py 8 5 192 192 120 160 >> gpurun_out/pmc_wg/time.log 2>&1
timeout -k 10 120 python tools/wgrad_probe.py 16 5 4 64 >> gpurun_out/pmc_wg/time.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES -d gpurun_out/pmc_wg/sq -o pmc --output-format csv -- python3 tools/wgrad_probe.py 8 2 > gpurun_out/pmc_wg/sq.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA -d gpurun_out/pmc_wg/lds -o pmc --output-format csv -- python3 tools/wgrad_probe.py 8 2 > gpurun_out/pmc_wg/lds.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_wg/fetch -o pmc --output-format csv -- python3 tools/wgrad_probe.py 8 2 > gpurun_out/pmc_wg/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o t -- python3 bench.py --workload train_kp --steps 3 --warmup 1 > gpurun_out/prof_train.log 2>&1
