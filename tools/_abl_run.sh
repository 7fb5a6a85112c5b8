set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_up4 -o u -- python3 tools/up4_probe.py 8 5 > gpurun_out/prof_up4.log 2>&1
