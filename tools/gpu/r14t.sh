#!/bin/bash
# e2e streams with two groups in flight (POSFEAT_EXTRACT_INFLIGHT=2) after the copy-stream D2H / prewarm changes
set -o pipefail
mkdir -p gpurun_out/r14t
export PYTHONUNBUFFERED=1
run() {  # tag sizes env...
  local tag=$1 sz=$2; shift 2
  env "$@" timeout -k 10 300 python -u tools/extract_e2e.py --sizes $sz --seqs 96 > gpurun_out/r14t/e2e_$tag.txt 2>&1 || { tail -20 gpurun_out/r14t/e2e_$tag.txt; return 1; }
  tail -1 gpurun_out/r14t/e2e_$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cold']; print('$tag', round(c['images_per_s'],1), 'replay', round(c['kernel_path_replay_images_per_s'],1), c['host'])"
}
run hp_i1 hpatches || exit 1
run hp_i2 hpatches POSFEAT_EXTRACT_INFLIGHT=2 || exit 1
run mixed_i1 mixed || exit 1
run mixed_i2 mixed POSFEAT_EXTRACT_INFLIGHT=2 || exit 1
run 480_i1 480x640 || exit 1
run 480_i2 480x640 POSFEAT_EXTRACT_INFLIGHT=2 || exit 1
