set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf6r.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r6t_bf6r.log 2>&1
ab() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r6t_$tag.json 2>/dev/null; }
ab d1 POSFEAT_X=0
ab g1 POSFEAT_GEMM_B256=1
ab d2 POSFEAT_X=0
ab g2 POSFEAT_GEMM_B256=1
POSFEAT_GEMM_B256=1 timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r6t_b256.txt 2>&1
timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r6t_def.txt 2>&1
exit 0
