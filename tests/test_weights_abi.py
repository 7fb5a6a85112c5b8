"""CPU tests: state-dict layout, BN folding / packing, and the C-ABI library
(loads, exports every symbol include/posfeat_hip.h declares, layer table
consistent with the reference parameter layout).  No GPU compute here."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import ROOT


def test_state_dict_layout():
    from posfeat_amd import weights
    bb = weights.backbone_param_shapes()
    hd = weights.head_param_shapes()
    assert len(bb) == 300 and len(hd) == 9          # SURVEY §5 checkpoint layout
    keys = [k for k, _ in bb]
    assert keys[0] == "firstconv.weight" and keys[-1] == "conv_fine.bn.num_batches_tracked"
    assert "layer3.5.conv3.weight" in keys and "upconv3.conv.conv.weight" in keys
    assert sum(int(np.prod(s)) for k, s in bb if not k.endswith(("running_mean", "running_var",
               "num_batches_tracked"))) == 20508992
    assert sum(int(np.prod(s)) for _, s in hd) == 628930


def test_seeded_recipe_is_deterministic():
    from posfeat_amd import weights
    a, _ = weights.seeded_state_dicts(0, as_torch=False)
    b, _ = weights.seeded_state_dicts(0, as_torch=False)
    c, _ = weights.seeded_state_dicts(1, as_torch=False)
    assert all(np.array_equal(a[k], b[k]) for k in a)
    assert not np.array_equal(a["firstconv.weight"], c["firstconv.weight"])


def test_bn_fold_matches_conv_bn():
    from posfeat_amd import weights
    bb, _ = weights.seeded_state_dicts(0)
    x = torch.randn(1, 512, 9, 11, dtype=torch.float64)
    w, b = weights.fold_conv(bb, "iconv2.conv.weight", "iconv2.conv.bias", "iconv2.bn")
    y_fold = F.conv2d(x, torch.from_numpy(w), torch.from_numpy(b), padding=1)
    p = "iconv2.bn."
    y_ref = F.batch_norm(F.conv2d(x, bb["iconv2.conv.weight"].double(),
                                  bb["iconv2.conv.bias"].double(), padding=1),
                         bb[p + "running_mean"].double(), bb[p + "running_var"].double(),
                         bb[p + "weight"].double(), bb[p + "bias"].double(), False, 0.0, 1e-5)
    assert torch.allclose(y_fold, y_ref, atol=1e-10)


def test_pack_layout_kh_kw_cin():
    from posfeat_amd import weights
    w = np.arange(2 * 3 * 3 * 3, dtype=np.float64).reshape(2, 3, 3, 3)
    wp, _ = weights.pack_conv(w, np.zeros(2))
    # cin padded to 4, K = 3*3*4 = 36 -> Kpad 64
    assert wp.shape == (2, 64)
    assert wp[1, (1 * 3 + 2) * 4 + 0] == w[1, 0, 1, 2]
    assert wp[1, (1 * 3 + 2) * 4 + 3] == 0.0
    assert np.all(wp[:, 36:] == 0)


def test_pack_layout_chunk_major():
    from posfeat_amd import weights
    w = np.random.RandomState(0).randn(3, 64, 3, 3)
    wp, _ = weights.pack_conv(w, np.zeros(3))
    assert wp.shape == (3, 576)
    # K index = ((c // 32) * 9 + kh * 3 + kw) * 32 + c % 32
    for (o, c, kh, kw) in [(0, 0, 0, 0), (2, 33, 1, 2), (1, 63, 2, 0), (2, 31, 2, 2)]:
        assert wp[o, ((c // 32) * 9 + kh * 3 + kw) * 32 + c % 32] == np.float32(w[o, c, kh, kw])


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "posfeat_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(posfeat_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from posfeat_amd import _lib
    L = _lib.lib()
    names = _header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(L, n), "missing export %s" % n
        assert n in _lib.SIGNATURES, "no ctypes signature for %s" % n


def test_abi_host_only_calls():
    from posfeat_amd import _lib
    L = _lib.lib()
    assert L.posfeat_abi_version() == 1
    assert L.posfeat_strerror(-1).decode().startswith("posfeat")
    assert L.posfeat_conv_packed_k(3, 7, 7) == 224 and L.posfeat_conv_packed_k(64, 3, 3) == 576
    n = ctypes.c_size_t()
    assert L.posfeat_detect_workspace(1, 480, 640, 2048, ctypes.byref(n)) == 0 and n.value > 0
    assert L.posfeat_detect_workspace(1, 2, 640, 2048, ctypes.byref(n)) != 0
    # invalid descriptors are rejected before any device work
    d = _lib.ConvDesc(n=1, h=8, w=8, cin=3, x_cstride=3, cout=8, kh=3, kw=3, stride=1, pad=1,
                      y_cstride=8, res_cstride=0, act=0)
    assert L.posfeat_conv2d_nhwc(ctypes.byref(d), ctypes.c_void_p(16), ctypes.c_void_p(16), None,
                                 None, ctypes.c_void_p(16), None) == -1
    # weight planes that would overlap (plane stride < cout x packed K) are
    # rejected before any device work
    d = _lib.ConvDesc(n=1, h=8, w=8, cin=64, x_cstride=64, cout=64, kh=1, kw=1, stride=1, pad=0,
                      y_cstride=64, res_cstride=0, act=0)
    kpad = L.posfeat_conv_packed_k(64, 1, 1)
    p = ctypes.c_void_p(256)
    assert L.posfeat_conv2d_nhwc_planes(ctypes.byref(d), p, p, p, 64 * kpad - 1, None, None, p,
                                        None, 0, -1, None) == -1
    assert L.posfeat_conv2d_nhwc_planes(ctypes.byref(d), p, p, p, 0, None, None, p, None, 0, -1,
                                        None) == -1


def test_engine_layer_table_matches_state_dicts():
    from posfeat_amd import _lib, weights
    specs = _lib.model_specs()
    bb = dict(weights.backbone_param_shapes())
    hd = dict(weights.head_param_shapes())
    conv_keys = set()
    for name, co, ci, kh, kw, wo, bo in specs:
        if name == "head.prelu":
            continue
        mod, wk, bk, bn = weights.conv_sources(name)
        sd = bb if mod == "backbone" else hd
        assert sd[wk] == (co, ci, kh, kw), name
        conv_keys.add(wk)
        if bn:
            assert sd[bn + ".running_var"] == (co,)
    # every conv weight of both state dicts is consumed exactly once
    all_conv = {k for k, s in list(bb.items()) + list(hd.items()) if len(s) == 4}
    assert conv_keys == all_conv
    blob = weights.pack_for_device(*weights.seeded_state_dicts(0), specs)
    assert blob.size <= _lib.lib().posfeat_model_weight_floats()
    assert np.isfinite(blob).all()


@pytest.mark.parametrize("lib", ["libposfeat_hip.so", "libposfeat_hip_ab.so"])
def test_isa_hazard_guard(lib):
    """tools/isa_check.py on the built gfx950 ISA of the shipped library and
    of the A/B build: conv_bf6d_kernel's counted waits (each step's B-plane DMA
    issued before its four A register loads, no vmcnt(0) drain between them);
    no MFMA reading a v_cvt_pk_bf16_f32 result without wait states; no
    in-place cross-half packed-fp32 op; no s_barrier crossed with the wave's
    own LDS accesses outstanding; no device-function call in a kernel.  Every
    one of these fails (none is only reported)."""
    import subprocess
    import sys
    path = os.path.join(ROOT, "posfeat_amd", lib)
    if not os.path.exists(path):
        pytest.skip("%s not built" % lib)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_check.py"), "--lib", path],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    for line in ("in-place cross-half packed-fp32 ops: 0 in 0 kernels",
                 "s_barrier with LDS accesses outstanding: 0 in []",
                 "device-function calls (s_swappc): 0"):
        assert line in r.stdout, r.stdout[-2000:]
