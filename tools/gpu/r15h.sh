#!/bin/bash
# f3 end-to-end extraction streams on the final sources (default settings)
set -o pipefail
o=gpurun_out/r15h; mkdir -p $o
export PYTHONUNBUFFERED=1
run() {  # tag sizes
  local tag=$1 sz=$2
  timeout -k 10 300 python -u tools/extract_e2e.py --sizes $sz --seqs 96 > $o/e2e_$tag.txt 2>&1 || { tail -20 $o/e2e_$tag.txt; return 1; }
  tail -1 $o/e2e_$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cold']; print('$tag', round(c['images_per_s'],1), 'replay', round(c['kernel_path_replay_images_per_s'],1), c['host'])"
}
run hpatches hpatches || exit 1
run mixed mixed || exit 1
run 480x640 480x640 || exit 1
