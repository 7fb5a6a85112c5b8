# round 5: wgrad staging roles remapped (LDS store conflicts), ordered split-K
# sums; train + extract tests, train_desc profile, f3 extraction runs
set -o pipefail
mkdir -p gpurun_out/r13j
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_model.py tests/test_gpu_train_fullsize.py tests/test_gpu_trainer_plugpoints.py \
  tests/test_gpu_repeat.py tests/test_gpu_extract.py \
  > gpurun_out/r13j/tests.txt 2>&1 || { tail -30 gpurun_out/r13j/tests.txt; exit 1; }
tail -2 gpurun_out/r13j/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r13j/prof -o td -- \
  python3 -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/r13j/bench_td.txt 2>&1 || { tail -20 gpurun_out/r13j/bench_td.txt; exit 1; }
grep '^{"metric' gpurun_out/r13j/bench_td.txt | cut -c1-200
run() {  # tag sizes env...
  local tag=$1 sz=$2; shift 2
  env "$@" timeout -k 10 300 python -u tools/extract_e2e.py --sizes $sz --seqs 96 $EXTRA > gpurun_out/r13j/e2e_$tag.txt 2>&1 || { tail -20 gpurun_out/r13j/e2e_$tag.txt; return 1; }
  tail -1 gpurun_out/r13j/e2e_$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cold']; print('$tag', round(c['images_per_s'],1), round(c.get('steady_images_per_s',0),1), 'replay', round(c['kernel_path_replay_images_per_s'],1), 'setup', round(c['setup_s'],2), c.get('reader'), c['host'])"
}
run mixed mixed || exit 1
run hp hpatches || exit 1
run mixed_loader mixed POSFEAT_EXTRACT_READER=loader || exit 1
run hp_nodb hpatches POSFEAT_TILE_DB=0 || exit 1
run 480 480x640 || exit 1
