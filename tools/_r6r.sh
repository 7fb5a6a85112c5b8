set -e
timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r6r.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6r.log 2>&1
bash tools/_r6s.sh
