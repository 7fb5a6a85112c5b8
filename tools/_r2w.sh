set -e
POSFEAT_BF6=1 POSFEAT_AUTOTUNE_LOG=1 timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r2w_bf6.log 2> gpurun_out/lt_r2w_bf6.err
