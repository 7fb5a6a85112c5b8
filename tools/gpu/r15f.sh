#!/bin/bash
# weight-gradient split heuristics, same-box A/B on train_desc (AB build knobs)
set -o pipefail
o=gpurun_out/r15f; mkdir -p $o
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
td() {  # tag env...
  local tag=$1; shift
  env POSFEAT_HIP_LIB=$AB "$@" timeout -k 10 300 python -u bench.py --workload train_desc --steps 10 --warmup 3 --no-cpu-baseline > $o/td_$tag.txt 2>&1 || { tail -20 $o/td_$tag.txt; return 1; }
  grep '^{"metric' $o/td_$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], {k: round(v, 2) for k, v in d['breakdown_ms'].items()} if isinstance(d.get('breakdown_ms'), dict) else '')"
}
td base || exit 1
td t2048 POSFEAT_WG_TARGET=2048 || exit 1
td m4 POSFEAT_WG_MINCH=4 || exit 1
td t2048m4 POSFEAT_WG_TARGET=2048 POSFEAT_WG_MINCH=4 || exit 1
td w4096 POSFEAT_WINO_WG_TARGET=4096 || exit 1
td w1024 POSFEAT_WINO_WG_TARGET=1024 || exit 1
td base2 || exit 1
