set -e
timeout -k 10 900 python -u -m pytest tests/test_gpu_trainer_plugpoints.py tests/test_train_kp.py tests/test_desc_grad.py tests/test_bb_train.py tests/test_gpu_correlation.py tests/test_gpu_api.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2r.log 2>&1
