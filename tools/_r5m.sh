set -e
# bf6b ablations (POSFEAT_ABL: 1 no MFMA, 2 no DMA, 4 no per-chunk wait/barrier, 8 no split);
# timing only -- results are garbage under any nonzero value
for v in 0 1 2 4 8 6 14 0; do
  POSFEAT_ABL=$v timeout -k 10 300 python tools/layer_timing.py 32 480 640 > gpurun_out/abl_r5m_$v.txt 2>&1
done
exit 0
