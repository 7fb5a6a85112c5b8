set -e
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6p.log 2>&1
timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r6p.txt 2>&1
bash tools/_r6o.sh
