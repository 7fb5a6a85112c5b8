set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf6r.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r6d_bf6r.log 2>&1
timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r6d.txt 2>&1
POSFEAT_WINO_IN2=0 timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r6d_in4.txt 2>&1
ab() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/bench_r6d_$tag.json 2>/dev/null; }
ab n1 POSFEAT_X=0
ab o1 POSFEAT_WINO_IN2=0
ab n2 POSFEAT_X=0
ab o2 POSFEAT_WINO_IN2=0
exit 0
