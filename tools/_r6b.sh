set -e
for v in 0 23 1; do
  POSFEAT_WINO_ENC=$v timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6b_enc$v.log 2>&1 || true
done
POSFEAT_BF6=0 timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6b_fp32.log 2>&1 || true
POSFEAT_BF6=0 POSFEAT_WINO_ENC=0 timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6b_fp32_enc0.log 2>&1 || true
exit 0
