set -e
ab() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_r6q_$tag.json 2>/dev/null; }
ab D3a POSFEAT_BF6D=3
ab D2a POSFEAT_BF6D=2
ab D4a POSFEAT_BF6D=4
ab D3b POSFEAT_BF6D=3
ab D2b POSFEAT_BF6D=2
ab D4b POSFEAT_BF6D=4
exit 0
