set -e
POSFEAT_EXTRACT_TRACE=1 timeout -k 10 400 python tools/extract_e2e.py > gpurun_out/e2e_r2p.json 2> gpurun_out/e2e_r2p.err
