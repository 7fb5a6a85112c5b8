#!/bin/bash
# round 6: full-size training vs fp64 (two fp32 realisations), side-stream
# ablations (A/B build, timing only), f3 e2e runs incl. Aachen
set -e
tag=r16d
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 600 $o/train_full.log python -u -m pytest tests/test_gpu_train_fullsize.py -m gpu -v -s --timeout 600 --timeout-method thread
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for abl in 0 1 2 4 7; do
  POSFEAT_HIP_LIB=$AB POSFEAT_SIDE_ABL=$abl $chk 300 $o/bench_side_abl$abl.log python bench.py --no-cpu-baseline --no-secondary --steps 30
done
$chk 600 $o/e2e_aachen.log python -u tools/extract_e2e.py --sizes aachen --seqs 24
$chk 400 $o/e2e_480.log python -u tools/extract_e2e.py --seqs 96
$chk 400 $o/e2e_hpatches.log python -u tools/extract_e2e.py --sizes hpatches --seqs 96
$chk 400 $o/e2e_mixed.log python -u tools/extract_e2e.py --sizes mixed --seqs 96
grep -E "passed|failed" $o/train_full.log | tail -2; grep -E "largest relative" $o/train_full.log | tail -1
for abl in 0 1 2 4 7; do echo "abl $abl: $(grep '^{' $o/bench_side_abl$abl.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
for f in aachen 480 hpatches mixed; do python3 -c "
import json; d=json.loads([l for l in open('$o/e2e_$f.log') if l.startswith('{')][-1])['cold']
print('$f', {k: round(v,3) if isinstance(v,float) else v for k,v in d.items() if k in ('images','images_per_s','images_per_s_incl_setup','setup_s','kernel_path_images_per_s','kernel_path_replay_images_per_s','whole_over_replay','whole_incl_setup_over_replay','group')})"; done
exit 0
