set -e
# counters on the head.conv2 probe -> traffic json, then the bench and its kernel trace
tools/pmc_conv2.sh gpurun_out/pmc3
python tools/traffic_json.py gpurun_out/pmc3 profiles/head_conv2_traffic.json 8 > gpurun_out/traffic.log
cp profiles/head_conv2_traffic.json gpurun_out/head_conv2_traffic.json
timeout -k 10 400 python bench.py > gpurun_out/bench_r1c.json 2> gpurun_out/bench_r1c.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_r1c -o b -- python3 bench.py --steps 5 --no-cpu-baseline > gpurun_out/prof_bench_r1c.log 2>&1
