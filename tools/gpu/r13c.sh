# round 5: GEMM probe (8-wave, A and B by LDS DMA) vs the 4-wave k16; f3 stream
# accounting with the shared weight store and workspace reservation
set -o pipefail
mkdir -p gpurun_out/r13c
export PYTHONUNBUFFERED=1
bash tools/probe/build.sh > gpurun_out/r13c/probe_build.txt 2>&1 || { tail gpurun_out/r13c/probe_build.txt; exit 1; }
timeout -k 10 120 ./probe_build/gemm_y 10 > gpurun_out/r13c/gemm_y.txt 2>&1 || { cat gpurun_out/r13c/gemm_y.txt; exit 1; }
cat gpurun_out/r13c/gemm_y.txt
timeout -k 10 120 ./probe_build/gemm_probe 10 > gpurun_out/r13c/gemm_probe.txt 2>&1 || exit 1
cat gpurun_out/r13c/gemm_probe.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_api.py tests/test_gpu_bench_config.py::test_engine_weight_cache_and_weights_changed > gpurun_out/r13c/tests.txt 2>&1 || { tail -30 gpurun_out/r13c/tests.txt; exit 1; }
tail -3 gpurun_out/r13c/tests.txt
for s in mixed hpatches; do
  for inf in 1 2; do
    POSFEAT_EXTRACT_INFLIGHT=$inf timeout -k 10 300 python -u tools/extract_e2e.py --sizes $s --seqs 96 > gpurun_out/r13c/e2e_${s}_inf$inf.txt 2>&1 || exit 1
    tail -1 gpurun_out/r13c/e2e_${s}_inf$inf.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cold']; print('$s inflight $inf', round(c['images_per_s'],1), round(c.get('steady_images_per_s',0),1), 'replay', round(c['kernel_path_replay_images_per_s'],1), 'setup', round(c['setup_s'],2), c['host'], c['engine_stats'])"
  done
done
