set -e
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_r5r.log 2>&1
ab() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r5r_$tag.json 2>/dev/null; }
ab d1 POSFEAT_X=0
ab n0 POSFEAT_GEMM_N64=0
ab d2 POSFEAT_X=0
ab old POSFEAT_HIP_LIB=$GRAFT_REPO_ROOT/posfeat_amd/libposfeat_hip_r5j.so
timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r5r.txt 2>&1
exit 0
