set -e
POSFEAT_BF6=1 POSFEAT_BF6_NST=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2z.log 2>&1
for n in 2 3 4; do
POSFEAT_BF6=1 POSFEAT_BF6_NST=$n timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r2z_nst$n.json 2>/dev/null
done
POSFEAT_BF6=1 POSFEAT_BF6_NST=4 timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r2z_nst4.log 2>&1
