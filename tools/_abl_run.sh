set -e
POSFEAT_AUTOTUNE_LOG=1 timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_tune.log 2> gpurun_out/tune.log
POSFEAT_AUTOTUNE=0 timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_notune.log 2>&1
