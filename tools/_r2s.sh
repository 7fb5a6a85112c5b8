set -e
timeout -k 10 900 python -u -m pytest tests/test_gpu_syncbn.py tests/test_bb_train.py tests/test_gpu_trainer_plugpoints.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2s.log 2>&1
