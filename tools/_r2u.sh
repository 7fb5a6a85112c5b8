set -e
for a in 0 1 2 3; do
POSFEAT_SIDE_AT=$a timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r2u_at$a.json 2>/dev/null
done
POSFEAT_SIDE_AT=2 timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r2u_at2.log 2>&1
