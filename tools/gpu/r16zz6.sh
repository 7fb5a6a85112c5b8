#!/bin/bash
# round 6: the f3 end-to-end runs (tools/extract_e2e.py, fresh processes) on
# the final sources (after the batched weight-stationary GEMMs): one size, HPatches sizes, mixed sizes, the Aachen layout
set -e
tag=r16zz6
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
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
