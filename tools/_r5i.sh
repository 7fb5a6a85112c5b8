set -e
POSFEAT_WINO_ENC=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_train_tap.py -v -s -k shape1 --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r5i_tap_enc0.log 2>&1 || true
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r5i.log 2>&1 || true
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/pmc_r5i -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline > gpurun_out/pmc_r5i.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_r5i2 -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline > gpurun_out/pmc_r5i2.log 2>&1
exit 0
