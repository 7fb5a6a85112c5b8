# round 5: per-layer timing of the extraction forward at B = 32 (HIP events)
set -o pipefail
mkdir -p gpurun_out/r13v
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/layer_timing.py 32 > gpurun_out/r13v/lt_b32.txt 2>&1 || { tail -20 gpurun_out/r13v/lt_b32.txt; exit 1; }
tail -5 gpurun_out/r13v/lt_b32.txt
