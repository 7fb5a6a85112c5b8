set -e
ab() { tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 "$@" > gpurun_out/bench_r6g_$tag.json 2>/dev/null; }
ab b32a --batch 32
ab b64a --batch 64
ab b32b --batch 32
ab b64b --batch 64
ab b48a --batch 48
ab b32c --batch 32
ab b64c --batch 64
exit 0
