T="tests/test_gpu_train_tap.py::test_traintap_backward"
for cfg in "X=1" "POSFEAT_WINO=0" "POSFEAT_BF6_HALO=0"; do
  env $cfg timeout -k 10 300 python -u -m pytest "$T" -m gpu -q -s --timeout 200 --timeout-method thread > "gpurun_out/tt_r4c_${cfg}.log" 2>&1
done
exit 0
