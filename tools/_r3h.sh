timeout -k 10 600 python -u -m pytest tests/test_gpu_train_tap.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3h3.log 2>&1
exit 0
