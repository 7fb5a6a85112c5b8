set -e
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_config.py tests/test_gpu_api.py tests/test_gpu_train_tap.py tests/test_train_kp.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3x.log 2>&1
for cfg in "X=1" "POSFEAT_IMGMOM_BLOCKS=120" "POSFEAT_IMGMOM_BLOCKS=16" "X=2"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 > "gpurun_out/bench_r3x_${cfg}.json" 2>/dev/null
done
