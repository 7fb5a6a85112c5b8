set -e
timeout -k 10 900 python -u -m pytest tests/test_train_kp.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2h.log 2>&1
timeout -k 10 120 python - > gpurun_out/match_timing_r2h.log 2>&1 <<'PY'
import sys, time, torch, numpy as np
sys.path.insert(0, '.')
from posfeat_amd import matchers as M
from oracle.match_ref import seeded_descriptors
for n in (2048, 8192):
    d1, d2 = seeded_descriptors(3, n, n)
    t1, t2 = torch.from_numpy(d1).cuda(), torch.from_numpy(d2).cuda()
    for _ in range(3): M.mnn_matcher(t1, t2)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(20): M.mnn_matcher(t1, t2)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 20
    print("n=%d mnn_matcher %.3f ms/call incl. D2H, sim %.1f GFLOP x2 passes" % (n, dt * 1e3, 2 * n * n * 128 / 1e9))
PY
timeout -k 10 300 python tools/bench_correlation.py > gpurun_out/bench_corr_r2h.log 2>&1
