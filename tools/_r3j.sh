set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf6r.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/gpu_tests_r3j.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r3j.json 2>/dev/null
POSFEAT_BF6R_NST=3 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r3j_nst3.json 2>/dev/null
POSFEAT_BF6R=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r3j_b.json 2>/dev/null
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r3j.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_tap.py tests/test_train_kp.py tests/test_gpu_trainer_plugpoints.py tests/test_gpu_train_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3i.log 2>&1
timeout -k 10 300 python bench.py --workload train_kp --no-cpu-baseline --steps 10 > gpurun_out/bench_kp_r3i.json 2> gpurun_out/bench_kp_r3i.err
