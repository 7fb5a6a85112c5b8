# f3: where the host time goes (staging / engine enqueue / detect), loader
# workers 4 vs 8, writers 4 vs 8, and the run without file writes
set -o pipefail
mkdir -p gpurun_out/r13d
export PYTHONUNBUFFERED=1
run() {  # tag sizes env...
  local tag=$1 sz=$2; shift 2
  env "$@" timeout -k 10 300 python -u tools/extract_e2e.py --sizes $sz --seqs 96 $EXTRA > gpurun_out/r13d/e2e_$tag.txt 2>&1 || return 1
  tail -1 gpurun_out/r13d/e2e_$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cold']; print('$tag', round(c['images_per_s'],1), round(c.get('steady_images_per_s',0),1), 'replay', round(c['kernel_path_replay_images_per_s'],1), 'setup', round(c['setup_s'],2), c['host'])"
}
run mixed_w4 mixed POSFEAT_EXTRACT_WORKERS=4 || exit 1
run mixed_w8 mixed POSFEAT_EXTRACT_WORKERS=8 || exit 1
run mixed_w8_wr8 mixed POSFEAT_EXTRACT_WORKERS=8 POSFEAT_EXTRACT_WRITERS=8 || exit 1
run hp_w4 hpatches POSFEAT_EXTRACT_WORKERS=4 || exit 1
run hp_w8 hpatches POSFEAT_EXTRACT_WORKERS=8 || exit 1
run hp_w12 hpatches POSFEAT_EXTRACT_WORKERS=12 POSFEAT_EXTRACT_WRITERS=8 || exit 1
EXTRA=--no-write run hp_w8_nowrite hpatches POSFEAT_EXTRACT_WORKERS=8 || exit 1
EXTRA=--no-write run mixed_w8_nowrite mixed POSFEAT_EXTRACT_WORKERS=8 || exit 1
nproc; python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
