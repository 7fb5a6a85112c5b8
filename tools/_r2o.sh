set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2o.log 2>&1
timeout -k 10 400 python tools/extract_e2e.py > gpurun_out/e2e_r2o.json 2> gpurun_out/e2e_r2o.err
