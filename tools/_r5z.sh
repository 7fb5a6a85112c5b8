set -e
# same-box A/B: this tree (bf6r + halo with amdgpu_waves_per_eu(2)) vs HEAD's library
ab() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/bench_r5z_$tag.json 2>/dev/null; }
ab new1 POSFEAT_X=0
ab head1 POSFEAT_HIP_LIB=$GRAFT_REPO_ROOT/posfeat_amd/libposfeat_hip_head.so
ab new2 POSFEAT_X=0
ab head2 POSFEAT_HIP_LIB=$GRAFT_REPO_ROOT/posfeat_amd/libposfeat_hip_head.so
ab new3 POSFEAT_X=0
ab head3 POSFEAT_HIP_LIB=$GRAFT_REPO_ROOT/posfeat_amd/libposfeat_hip_head.so
exit 0
