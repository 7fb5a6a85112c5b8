# round 5 f3 on the F(6x6) build: tile database regenerated, extract tests, e2e streams
set -o pipefail
mkdir -p gpurun_out/r13s
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u tools/tile_db.py records/tile_db.txt > gpurun_out/r13s/tile_db.log 2>&1 || { tail -20 gpurun_out/r13s/tile_db.log; exit 1; }
tail -3 gpurun_out/r13s/tile_db.log
cp records/tile_db.txt gpurun_out/r13s/tile_db.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_extract.py > gpurun_out/r13s/tests.txt 2>&1 || { tail -30 gpurun_out/r13s/tests.txt; exit 1; }
tail -3 gpurun_out/r13s/tests.txt
run() {  # tag sizes env...
  local tag=$1 sz=$2; shift 2
  env "$@" timeout -k 10 300 python -u tools/extract_e2e.py --sizes $sz --seqs 96 $EXTRA > gpurun_out/r13s/e2e_$tag.txt 2>&1 || { tail -20 gpurun_out/r13s/e2e_$tag.txt; return 1; }
  tail -1 gpurun_out/r13s/e2e_$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cold']; print('$tag', round(c['images_per_s'],1), round(c.get('steady_images_per_s',0),1), 'replay', round(c['kernel_path_replay_images_per_s'],1), 'setup', round(c['setup_s'],2), c.get('reader'), c['host'])"
}
run mixed mixed || exit 1
run hp hpatches || exit 1
run mixed_loader mixed POSFEAT_EXTRACT_READER=loader || exit 1
run hp_nodb hpatches POSFEAT_TILE_DB=0 || exit 1
run 480 480x640 || exit 1
EXTRA=--no-write run hp_nowrite hpatches || exit 1
