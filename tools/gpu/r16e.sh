#!/bin/bash
# round 6: LDS-staged gfuse_weights + two-pass MFMA border ring (side stream);
# F(6x6) variant tests; head / extraction parity; bench; Aachen e2e
set -e
tag=r16e
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
$chk 900 $o/tests.log python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_api.py tests/test_gpu_bench_config.py tests/test_gpu_extract.py tests/test_gpu_repeat.py -m gpu -q -rf --timeout 600 --timeout-method thread
$chk 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
$chk 300 $o/bench.log python bench.py --no-cpu-baseline --no-secondary --steps 40
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
for abl in 0 7; do
  POSFEAT_HIP_LIB=$AB POSFEAT_SIDE_ABL=$abl $chk 300 $o/bench_side_abl$abl.log python bench.py --no-cpu-baseline --no-secondary --steps 40
done
$chk 200 $o/lt.log python -u tools/layer_timing.py 32
$chk 900 $o/e2e_aachen.log python -u tools/extract_e2e.py --sizes aachen --seqs 24
tail -3 $o/tests.log; grep smoke $o/smoke.log
for f in bench bench_side_abl0 bench_side_abl7; do echo "$f: $(grep '^{' $o/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
grep -E "main stream|side:" $o/lt.log
python3 -c "
import json; d=json.loads([l for l in open('$o/e2e_aachen.log') if l.startswith('{')][-1])['cold']
print('aachen', {k: round(v,3) if isinstance(v,float) else v for k,v in d.items() if k in ('images','images_per_s','images_per_s_incl_setup','setup_s','kernel_path_images_per_s','kernel_path_replay_images_per_s','whole_over_replay','whole_incl_setup_over_replay','group','engine_workspace_mb')})"
exit 0
