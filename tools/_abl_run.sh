set -e
for k in halo glds; do
  echo "kernel: $k" >> gpurun_out/abl4.log
  POSFEAT_CONV_KERNEL=$k timeout -k 10 120 python tools/conv2_probe.py 8 5 >> gpurun_out/abl4.log 2>&1
done
POSFEAT_CONV_TILE=12 timeout -k 10 120 python tools/conv2_probe.py 8 5 >> gpurun_out/abl4.log 2>&1
POSFEAT_CONV_KERNEL=glds timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_glds.log 2>&1
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_halo.log 2>&1
