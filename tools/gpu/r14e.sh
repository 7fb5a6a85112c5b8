#!/bin/bash
# results D2H on a copy stream + pinned host memory prewarmed at construction: extract tests and e2e streams
set -o pipefail
mkdir -p gpurun_out/r14e
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_extract.py > gpurun_out/r14e/tests.txt 2>&1 || { tail -30 gpurun_out/r14e/tests.txt; exit 1; }
tail -2 gpurun_out/r14e/tests.txt
run() {  # tag sizes env...
  local tag=$1 sz=$2; shift 2
  env "$@" timeout -k 10 300 python -u tools/extract_e2e.py --sizes $sz --seqs 96 $EXTRA > gpurun_out/r14e/e2e_$tag.txt 2>&1 || { tail -20 gpurun_out/r14e/e2e_$tag.txt; return 1; }
  tail -1 gpurun_out/r14e/e2e_$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cold']; print('$tag', round(c['images_per_s'],1), round(c.get('steady_images_per_s',0),1), 'replay', round(c['kernel_path_replay_images_per_s'],1), 'setup', round(c['setup_s'],2), c.get('reader'), c['host'])"
}
run hp hpatches || exit 1
run mixed mixed || exit 1
run 480 480x640 || exit 1
EXTRA=--no-write run hp_nowrite hpatches || exit 1
