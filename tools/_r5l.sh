set -e
# same-box A/B: r5j library (DMA overlap in bf6b only) vs this tree (all ring kernels)
ab() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r5l_$tag.json 2>/dev/null; }
ab new0 POSFEAT_X=0
ab old0 POSFEAT_HIP_LIB=$GRAFT_REPO_ROOT/posfeat_amd/libposfeat_hip_r5j.so
ab new1 POSFEAT_X=0
ab old1 POSFEAT_HIP_LIB=$GRAFT_REPO_ROOT/posfeat_amd/libposfeat_hip_r5j.so
POSFEAT_HIP_LIB=$GRAFT_REPO_ROOT/posfeat_amd/libposfeat_hip_r5j.so timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/layer_timing_b32_r5l_old.txt 2>&1
timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/layer_timing_b32_r5l_new.txt 2>&1
exit 0
