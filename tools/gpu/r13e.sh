# round 5: ring kernel parity + headline bench + descriptor-training per-layer
# breakdown, then the f3 host-time sweep (tools/gpu/r13d.sh)
set -o pipefail
mkdir -p gpurun_out/r13e
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench_config.py tests/test_gpu_model.py tests/test_gpu_repeat.py > gpurun_out/r13e/tests.txt 2>&1 || { tail -30 gpurun_out/r13e/tests.txt; exit 1; }
tail -3 gpurun_out/r13e/tests.txt
timeout -k 10 300 python -u bench.py > gpurun_out/r13e/bench.json 2> gpurun_out/r13e/bench.err || { tail -20 gpurun_out/r13e/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r13e/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['roofline']['frac'], d['roofline_hbm']['label'], d['roofline_hbm']['avg_launch_ms'], d['conv_total'], {k: v['value'] for k, v in d['secondary_workloads'].items()})"
timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 > gpurun_out/r13e/train_desc.json 2> gpurun_out/r13e/train_desc.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/r13e/train_desc.json').read().strip().splitlines()[-1]); print('train_desc', d['value'], d['breakdown_ms']); [print(x) for x in d['top_conv_layers']]"
bash tools/gpu/r13d.sh
