"""Switches whose two forms must give BIT-identical engine outputs.

conv_bf6d_kernel (pre-split weights, A prefetched D chunks ahead in registers,
the default for the non-dense convs; the dense ones with POSFEAT_BF6X=0) against conv_bf6b_kernel (A staged through LDS, POSFEAT_BF6D=0):
the same bf16x6 products in the same order, so the engine's outputs must be
BIT-identical for every D (the switch is read once per process: each run is a
child process).  The B=8 480x640 bench instance covers the batched Winograd
GEMMs, the tap GEMM and the 1x1 / strided encoder convs (masked taps: the
register-A candidates TILE_BF6R_*)."""
import os
import subprocess
import sys

import numpy as np

from conftest import ab_env
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODE = r"""
import sys, numpy as np, torch
sys.path.insert(0, %(root)r)
from posfeat_amd.engine import ExtractionEngine
from posfeat_amd.weights import seeded_image, seeded_state_dicts
bb, hd = seeded_state_dicts(0)
eng = ExtractionEngine(bb, hd, device="cuda:0")
img = torch.from_numpy(np.stack([seeded_image(60 + i, 480, 640) for i in range(8)])).cuda()
r = eng.run(img, outputs=("local_map", "global_map"))
torch.cuda.synchronize()
np.savez(%(out)r, lp=r["local_point"].cpu().numpy(), lm=r["local_map"].cpu().numpy(),
         gm=r["global_map"].cpu().numpy())
"""


def _run(tmp_path, env_extra, tag):
    out = str(tmp_path / ("%s.npz" % tag))
    env = dict(os.environ, **ab_env(), **env_extra)   # the switches need the A/B build
    subprocess.run([sys.executable, "-c", CODE % {"root": ROOT, "out": out}], env=env,
                   check=True, timeout=240)
    return np.load(out)


def test_fused_upsample_bit_identical(tmp_path):
    """the decoder's x2 upsample interpolated inside the Winograd input
    transform (pf_up2ac_at: the upsample kernel's own arithmetic) equals the
    materialised upsample + transform (POSFEAT_UP2FUSE=0) bit for bit"""
    ref = _run(tmp_path, {"POSFEAT_UP2FUSE": "0"}, "u0")
    got = _run(tmp_path, {"POSFEAT_UP2FUSE": "1"}, "u1")
    for k in ("lp", "lm", "gm"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def test_bf6d_bit_identical_to_bf6b(tmp_path):
    """D = 2 (default), 3 and 4, the register-A candidates forced on every conv
    they serve (POSFEAT_CONV_TILE 26 = TILE_BF6R_128x128), and the 8-wave
    256x128 pre-split tile (TILE_BF6B_256x128 = 28: an autotuner candidate for
    the 1x1 convs, forced everywhere it is legal, and on the batched Winograd
    GEMMs via POSFEAT_GEMM_B256; D capped at 3 there)"""
    # the dense GEMMs / 1x1 convs run the 32x32x16 family here (POSFEAT_BF6X=0):
    # the 16x16x32 default is checked in test_gpu_bf6x.py
    x0 = {"POSFEAT_BF6X": "0"}
    ref = _run(tmp_path, dict(x0, POSFEAT_BF6D="0"), "b")   # LDS-staged bf6b
    for tag, env in (("d2", {}),                       # the default: deep A prefetch, D = 2
                     ("d3", {"POSFEAT_BF6D": "3"}),
                     ("d4", {"POSFEAT_BF6D": "4"}),
                     ("r26", {"POSFEAT_CONV_TILE": "26"}),
                     ("b256", {"POSFEAT_CONV_TILE": "28", "POSFEAT_GEMM_B256": "1"}),
                     ("b256d4", {"POSFEAT_CONV_TILE": "28", "POSFEAT_GEMM_B256": "1",
                                 "POSFEAT_BF6D": "4"})):
        got = _run(tmp_path, dict(x0, **env), tag)
        for k in ("lp", "lm", "gm"):
            np.testing.assert_array_equal(got[k], ref[k], err_msg="%s %s" % (tag, k))
    # conv precision mode 2: the Winograd / tap GEMM A operands pre-split by
    # their producers (conv_bf6s_kernel).  Its V planes exist for F(4x4) only,
    # so mode 2 runs the decoder on F(4x4): compared with the bf6b reference
    # on F(4x4) (POSFEAT_WINO6=0)
    ref4 = _run(tmp_path, dict(x0, POSFEAT_BF6D="0", POSFEAT_WINO6="0"), "b4")
    got = _run(tmp_path, dict(x0, POSFEAT_BF6="2"), "mode2")
    for k in ("lp", "lm", "gm"):
        np.testing.assert_array_equal(got[k], ref4[k], err_msg="mode2 %s" % k)
