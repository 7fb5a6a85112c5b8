for cfg in "X=1" "POSFEAT_WINO=0" "POSFEAT_BF6_HALO=0" "POSFEAT_BF6=0"; do
  env $cfg timeout -k 10 300 python -u -m pytest "tests/test_gpu_trainer_plugpoints.py::test_backbone_training_backward_vs_reference" -m gpu -q -s --timeout 200 --timeout-method thread > "gpurun_out/bbgrad_r3l_${cfg}.log" 2>&1
done
exit 0
