set -e
# counters on the dominant kernel (probe) -> traffic json, then the bench and its kernel trace
PROBE=tools/up4_probe.py tools/pmc_conv2.sh gpurun_out/pmc_up4e
python tools/traffic_json.py gpurun_out/pmc_up4e profiles/up4_traffic.json 8 conv_up4_kernel > gpurun_out/traffic_up4.log
cp profiles/up4_traffic.json gpurun_out/up4_traffic.json
timeout -k 10 400 python bench.py > gpurun_out/bench_r1d.json 2> gpurun_out/bench_r1d.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_r1d -o b -- python3 bench.py --steps 5 --no-cpu-baseline > gpurun_out/prof_bench_r1d.log 2>&1
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_r1d.log 2>&1
