set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_persistent.py -x -v --timeout 100 --timeout-method thread > gpurun_out/gpu_tests_r5q_persist.log 2>&1
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_r5q.log 2>&1
ab() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r5q_$tag.json 2>/dev/null; }
ab p1a POSFEAT_X=0
ab p0a POSFEAT_BF6P=0
ab p1b POSFEAT_X=0
ab p0b POSFEAT_BF6P=0
timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r5q.txt 2>&1
exit 0
