set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_up4d -o u -- python3 tools/up4_probe.py 8 5 > gpurun_out/prof_up4d.log 2>&1
timeout -k 10 300 python tools/layer_timing.py 8 480 640 > gpurun_out/lt_up4d.log 2>&1
