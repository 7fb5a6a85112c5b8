set -e
for cfg in "X=1" "POSFEAT_SIDE_AT=1" "POSFEAT_SIDE_AT=3" "POSFEAT_SIDE=0" "X=2"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 > "gpurun_out/bench_r3q_${cfg}.json" 2>/dev/null
done
