set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf6r.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r6k.log 2>&1
ab() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r6k_$tag.json 2>/dev/null; }
ab d1 POSFEAT_X=0
ab D2 POSFEAT_BF6D=2
ab D3 POSFEAT_BF6D=3
ab D4 POSFEAT_BF6D=4
ab d2 POSFEAT_X=0
ab D3b POSFEAT_BF6D=3
POSFEAT_BF6D=3 timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r6k_d3.txt 2>&1
timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r6k_def.txt 2>&1
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r6k_full.log 2>&1 || true
exit 0
