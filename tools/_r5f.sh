set -e
POSFEAT_WINO_ENC=1 timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/layer_timing_b32_winoenc_r5f.txt 2>&1
POSFEAT_WINO_ENC=1 timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/layer_timing_b8_winoenc_r5f.txt 2>&1
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/layer_timing_b8_r5f.txt 2>&1
exit 0
