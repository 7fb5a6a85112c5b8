set -o pipefail
mkdir -p gpurun_out/r13b
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_repeat.py tests/test_gpu_correlation.py::test_disk_flash_matches_dense_path tests/test_gpu_train_tap.py > gpurun_out/r13b/tests.txt 2>&1 || { tail -30 gpurun_out/r13b/tests.txt; exit 1; }
tail -5 gpurun_out/r13b/tests.txt
POSFEAT_EXTRACT_TRACE=1 timeout -k 10 300 python -u tools/extract_e2e.py --sizes hpatches --seqs 96 > gpurun_out/r13b/hp_trace.txt 2>&1 || exit 1
tail -c 600 gpurun_out/r13b/hp_trace.txt
POSFEAT_ENGINE_MAX_SHAPES=128 timeout -k 10 300 python -u tools/extract_e2e.py --sizes hpatches --seqs 96 > gpurun_out/r13b/hp_nolru.txt 2>&1 || exit 1
POSFEAT_AUTOTUNE=0 timeout -k 10 300 python -u tools/extract_e2e.py --sizes hpatches --seqs 96 > gpurun_out/r13b/hp_noat.txt 2>&1 || exit 1
POSFEAT_EXTRACT_TRACE=1 timeout -k 10 300 python -u tools/extract_e2e.py --sizes mixed --seqs 96 > gpurun_out/r13b/mixed_trace.txt 2>&1 || exit 1
for f in hp_nolru hp_noat mixed_trace; do tail -1 gpurun_out/r13b/$f.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cold']; print('$f', round(c['images_per_s'],1), round(c.get('steady_images_per_s',0),1), round(c['kernel_path_replay_images_per_s'],1), c['engine_stats'])"; done
