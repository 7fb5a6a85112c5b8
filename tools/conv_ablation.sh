#!/bin/bash
# Build PF_PROBE ablation variants of the conv kernel (see conv.hip) into
# probe_build/ (built here; time each on the box with tools/conv2_probe.py
# under POSFEAT_HIP_LIB=probe_build/libposfeat_probeN.so).
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
out="$root/probe_build"; mkdir -p "$out"
objs=$(ls "$root"/build/obj/*.o | grep -v '/conv.o$')
for v in ${PROBES:-0 1 2 3 4}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DPF_PROBE=$v \
    -c "$root/posfeat_amd/csrc/conv.hip" -o "$out/conv_$v.o"
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "$out/conv_$v.o" $objs \
    -o "$out/libposfeat_probe$v.so"
done
