set -e
# same box: decoder Winograd GEMMs on bf6b (LDS A) vs bf6r (A in registers, B ring 2/3) after the DMA-overlap fix
run() { tag=$1; shift; env "$@" timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/lt_r5n_$tag.txt 2>&1; }
run def POSFEAT_X=0
run r2 POSFEAT_BF6R=1 POSFEAT_BF6R_NST=2
run r3 POSFEAT_BF6R=1 POSFEAT_BF6R_NST=3
run def2 POSFEAT_X=0
exit 0
