set -e
timeout -k 10 600 python -u -m pytest tests/test_train_kp.py tests/test_bb_train.py tests/test_desc_grad.py tests/test_gpu_trainer_plugpoints.py tests/test_gpu_train_tap.py -m gpu -q -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4a.log 2>&1 || true
timeout -k 10 300 python bench.py --workload train_desc --no-cpu-baseline --steps 10 > gpurun_out/bench_desc_r4a.json 2>/dev/null
POSFEAT_WGRAD_BF6=0 timeout -k 10 300 python bench.py --workload train_desc --no-cpu-baseline --steps 10 > gpurun_out/bench_desc_r4a_off.json 2>/dev/null
timeout -k 10 300 python bench.py --workload train_kp --no-cpu-baseline --steps 10 > gpurun_out/bench_kp_r4a.json 2>/dev/null
