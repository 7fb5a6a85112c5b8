set -e
timeout -k 10 400 python tools/extract_e2e.py > gpurun_out/e2e_r2q.json 2> gpurun_out/e2e_r2q.err
timeout -k 10 400 python tools/extract_e2e.py --timing > gpurun_out/e2e_r2q_serial.json 2> gpurun_out/e2e_r2q_serial.err
