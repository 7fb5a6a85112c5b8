set -e
timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r5s.txt 2>&1
POSFEAT_GEMM_N64=0 timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r5s_n0.txt 2>&1
exit 0
