#!/bin/bash
# round 6: (1) A/B the 128 x 64 dense / stem plans on 256 x 64 tiles
# (POSFEAT_BF6X_RB4N64=1): parity on the model tests, layer timing;
# (2) the f3 end-to-end runs on the current sources (keypoint selection,
# conv3 + downsample GEMM, deferred seeded weights)
set -e
tag=r16w
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
POSFEAT_HIP_LIB=$AB POSFEAT_BF6X_RB4N64=1 $chk 400 $o/tests_rb4.log python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_config.py -m gpu -q -rf --timeout 300 --timeout-method thread
tail -2 $o/tests_rb4.log
for p in 1 2; do for v in base rb4; do
  case $v in base) e="";; rb4) e="POSFEAT_BF6X_RB4N64=1";; esac
  env POSFEAT_HIP_LIB=$AB $e $chk 200 $o/lt_${v}_$p.log python -u tools/layer_timing.py 32
done; done
for f in $o/lt_*.log; do echo "== $f $(grep 'main stream' $f | cut -c1-40)"; grep -E "conv:(firstconv|layer1\.[12]\.conv1|layer1\.0\.conv1|conv_fine) " $f; done
$chk 400 $o/e2e_480.log python -u tools/extract_e2e.py --seqs 96
$chk 400 $o/e2e_hpatches.log python -u tools/extract_e2e.py --sizes hpatches --seqs 96
$chk 400 $o/e2e_mixed.log python -u tools/extract_e2e.py --sizes mixed --seqs 96
$chk 600 $o/e2e_aachen.log python -u tools/extract_e2e.py --sizes aachen --seqs 24
for f in $o/e2e_*.log; do python3 - "$f" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith('{'):
        c = json.loads(line)['cold']
        print(sys.argv[1].split('/')[-1], {k: (round(c[k], 3) if isinstance(c[k], float) else c[k]) for k in c if 'per_s' in k or 'over' in k or k in ('setup_s', 'images', 'setup_phases_s')})
PY
done
exit 0
