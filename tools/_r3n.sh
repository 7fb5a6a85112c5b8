set -e
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 > gpurun_out/bench_r3n.json 2>gpurun_out/bench_r3n.err
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 --no-graph > gpurun_out/bench_r3n_eager.json 2>>gpurun_out/bench_r3n.err
