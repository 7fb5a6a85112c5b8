timeout -k 10 900 python -u -m pytest tests/test_train_kp.py tests/test_bb_train.py tests/test_desc_grad.py tests/test_gpu_trainer_plugpoints.py tests/test_gpu_train_tap.py tests/test_gpu_train_fullsize.py tests/test_gpu_syncbn.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4e.log 2>&1
timeout -k 10 300 python bench.py --workload train_kp --no-cpu-baseline --steps 10 > gpurun_out/bench_kp_r4e.json 2>/dev/null
POSFEAT_WGRAD_BF6_ALL=0 timeout -k 10 300 python bench.py --workload train_kp --no-cpu-baseline --steps 10 > gpurun_out/bench_kp_r4e_off.json 2>/dev/null
timeout -k 10 300 python bench.py --workload train_desc --no-cpu-baseline --steps 10 > gpurun_out/bench_desc_r4e.json 2>/dev/null
POSFEAT_WGRAD_BF6_ALL=0 timeout -k 10 300 python bench.py --workload train_desc --no-cpu-baseline --steps 10 > gpurun_out/bench_desc_r4e_off.json 2>/dev/null
exit 0
