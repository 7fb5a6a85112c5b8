set -e
for a in 0 1 2 3; do
POSFEAT_ABL=$a timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r3c_abl$a.log 2>&1
done
POSFEAT_BF6=0 POSFEAT_ABL=1 timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r3c_fp32_abl1.log 2>&1
POSFEAT_BF6=0 POSFEAT_ABL=0 timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r3c_fp32_abl0.log 2>&1
