#!/bin/bash
# round 6: gcombine's y staging with swizzled column slots (half-waves on
# opposite bank halves): the tests that run it, LDS bank conflicts (one PMC
# pass), layer timing x2
set -e
tag=r16zj
o=gpurun_out/$tag
mkdir -p "$o"
chk=tools/gpu_check.sh
export PYTHONUNBUFFERED=1
AB=$PWD/posfeat_amd/libposfeat_hip_ab.so
$chk 600 $o/tests.log python -u -m pytest tests/test_gpu_bench_config.py tests/test_gpu_repeat.py tests/test_gpu_fusions.py -m gpu -q -rf --timeout 300 --timeout-method thread
tail -2 $o/tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d $o/pmc -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline --no-secondary > $o/pmc.log 2>&1 || exit 100
f=$(find $o/pmc -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY' | tee $o/pmc_summary.txt
import csv, sys, collections
d = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if "gemm_ws" in k or "up4tap_gcombine" in k:
        key = k.split("(")[0][:60] + " " + r["Grid_Size"]
        d[key][r["Counter_Name"]] += float(r["Counter_Value"]); n[(key, r["Counter_Name"])] += 1
for key, c in d.items():
    m = {k: v / max(1, n[(key, k)]) for k, v in c.items()}
    wc = m.get("SQ_WAVE_CYCLES", 1)
    print(key, {k: round(v) for k, v in m.items()})
    print("   wait %.2f  inst-stall %.2f  issuing %.2f  lds-conflict/idx %.3f" % (
        m.get("SQ_WAIT_ANY", 0) / wc, m.get("SQ_WAIT_INST_ANY", 0) / wc,
        m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        m.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, m.get("SQ_LDS_IDX_ACTIVE", 1))))
PY
rm -rf $o/pmc
for p in 1 2; do
  $chk 200 $o/lt_$p.log python -u tools/layer_timing.py 32
done
for p in 1 2; do echo "== $p $(grep 'main stream' $o/lt_$p.log | cut -c1-40)"; grep -E "gcombine|up4tap" $o/lt_$p.log; done
exit 0
