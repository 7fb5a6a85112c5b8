for cfg in "POSFEAT_BF6_HALO=0" "POSFEAT_BF6=0" "POSFEAT_BF6R=0" "X=1"; do
  env $cfg timeout -k 10 300 python -u -m pytest "tests/test_gpu_trainer_plugpoints.py::test_backbone_training_backward_vs_reference" tests/test_bb_train.py -m gpu -q --timeout 200 --timeout-method thread > "gpurun_out/bbgrad_r3k_${cfg}.log" 2>&1
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_tap.py tests/test_train_kp.py tests/test_gpu_trainer_plugpoints.py tests/test_gpu_train_fullsize.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3k.log 2>&1
timeout -k 10 300 python bench.py --workload train_kp --no-cpu-baseline --steps 10 > gpurun_out/bench_kp_r3k.json 2> gpurun_out/bench_kp_r3k.err
timeout -k 10 300 python bench.py --workload train_desc --no-cpu-baseline --steps 10 > gpurun_out/bench_desc_r3k.json 2> gpurun_out/bench_desc_r3k.err
exit 0
