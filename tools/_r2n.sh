set -e
timeout -k 10 400 python tools/extract_e2e.py --timing > gpurun_out/e2e_r2n_timing.json 2> gpurun_out/e2e_r2n_timing.err
timeout -k 10 400 python tools/extract_e2e.py > gpurun_out/e2e_r2n.json 2> gpurun_out/e2e_r2n.err
