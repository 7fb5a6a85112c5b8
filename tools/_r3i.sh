set -e
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_tap.py tests/test_train_kp.py tests/test_gpu_trainer_plugpoints.py tests/test_gpu_train_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3i.log 2>&1
timeout -k 10 300 python bench.py --workload train_kp --no-cpu-baseline --steps 10 > gpurun_out/bench_kp_r3i.json 2> gpurun_out/bench_kp_r3i.err
POSFEAT_SIDE=0 timeout -k 10 300 python bench.py --workload train_kp --no-cpu-baseline --steps 10 > gpurun_out/bench_kp_r3i_noside.json 2> gpurun_out/bench_kp_r3i.err
