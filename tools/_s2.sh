set -e
timeout -k 10 300 python -u -m pytest tests/test_bb_train.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/s2_tests.log 2>&1
timeout -k 10 300 python bench.py --workload train_desc --steps 10 --warmup 3 > gpurun_out/bench_desc.json 2> gpurun_out/bench_desc.err
POSFEAT_S2PHASE=0 timeout -k 10 300 python bench.py --workload train_desc --steps 10 --warmup 3 > gpurun_out/bench_desc_zi.json 2>> gpurun_out/bench_desc.err
