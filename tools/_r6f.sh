set -e
timeout -k 10 600 python -u tools/stem_tiles.py > gpurun_out/stem_tiles_r6f.log 2>&1
exit 0
