set -e
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_fullsize.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/gpu_tests_r2t.log 2>&1
timeout -k 10 300 python bench.py --workload train_kp --steps 10 --warmup 3 > gpurun_out/bench_train_kp_r2t.json 2> gpurun_out/bench_train_kp_r2t.err
timeout -k 10 300 python bench.py --workload train_desc --steps 10 --warmup 3 > gpurun_out/bench_train_desc_r2t.json 2> gpurun_out/bench_train_desc_r2t.err
