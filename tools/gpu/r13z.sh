# round 5: side stream + events shared by the engine instances (no stream create / destroy per shape)
set -o pipefail
mkdir -p gpurun_out/r13z
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_bench_config.py tests/test_gpu_model.py > gpurun_out/r13z/tests.txt 2>&1 || { tail -30 gpurun_out/r13z/tests.txt; exit 1; }
tail -2 gpurun_out/r13z/tests.txt
run() {  # tag sizes env...
  local tag=$1 sz=$2; shift 2
  env "$@" timeout -k 10 300 python -u tools/extract_e2e.py --sizes $sz --seqs 96 > gpurun_out/r13z/e2e_$tag.txt 2>&1 || { tail -20 gpurun_out/r13z/e2e_$tag.txt; return 1; }
  tail -1 gpurun_out/r13z/e2e_$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cold']; print('$tag', round(c['images_per_s'],1), round(c.get('steady_images_per_s',0),1), 'replay', round(c['kernel_path_replay_images_per_s'],1), c['host'])"
}
run hp hpatches || exit 1
run mixed mixed || exit 1
run 480 480x640 || exit 1
