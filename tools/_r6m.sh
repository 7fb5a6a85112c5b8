set -e
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r6m.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6m.log 2>&1
timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r6m.txt 2>&1
bash tools/_r6l.sh
