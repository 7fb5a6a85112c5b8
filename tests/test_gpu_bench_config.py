"""Parity at the benchmarked configuration and at real-data shapes.

* The bench runs one engine instance at B=32 (bench.EXTRACT_BATCH; B=8 in
  round 1), 480x640, autotuned on its first forward (bench.py).  Here the same instance (fresh engine, autotune on, side
  stream on) is compared image by image with B=1 runs and with the torch-CPU
  oracle: local_point within 1e-4 absolute, local_map within 1e-5 of its
  scale (tests/tol.py) and the batched detector's keypoints
  identical to the per-image detector's, except at near-ties of the map.
* Aachen-like shapes that are not 480x640 (768x1024, and 496x656 whose H/8 and
  W/8 are not multiples of 4, so the decoder takes the Winograd F(2x2) path and
  H/16, W/16 are odd) run end to end against the oracle with the Aachen
  detector configuration (configs/extract_aachen.yaml: nms_radius 3, thr 0.5).
* The engine's non-default paths behind environment switches (POSFEAT_SIDE=0:
  serial image branch; POSFEAT_UP4TAP=0: head.conv2's upsampled part as the
  low-res Winograd F(4x4) conv; POSFEAT_UP4WINO=0 with it: by bilinear phases;
  POSFEAT_IMGSTATS=0: convimg's instance-norm statistics from the convimg conv
  instead of the image's tap moments) agree with the default engine (SIDE:
  bit-identical; the others: tests/tol.py's bounds).  (POSFEAT_DISK_FLASH does not touch the
  extraction engine: a no-op guard here, the DiskLoss A/B is in
  test_gpu_correlation.py.)
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import tol
from conftest import ROOT

pytestmark = pytest.mark.gpu

TOL = 1e-4   # coordinates, scores and descriptors at the keypoints (absolute)


def _maxerr(a, b):
    a = a.detach().cpu().double() if torch.is_tensor(a) else torch.from_numpy(np.asarray(a)).double()
    b = b.detach().cpu().double() if torch.is_tensor(b) else torch.from_numpy(np.asarray(b)).double()
    return float((a - b).abs().max()), max(1.0, float(b.abs().max()))


def _new_engine(dev):
    from posfeat_amd.engine import ExtractionEngine
    from posfeat_amd.weights import seeded_state_dicts
    bb, hd = seeded_state_dicts(0)
    return ExtractionEngine(bb, hd, device=dev)


# A/B comparisons run in a child process on the A/B build (the shipped
# library ignores the path switches): the default path and the switched one,
# each on a fresh engine instance (the switches are read when an instance is
# planned), same inputs
AB_CHILD = r"""
import os, sys, numpy as np, torch
sys.path.insert(0, %(root)r)
from posfeat_amd.engine import ExtractionEngine
from posfeat_amd.weights import seeded_state_dicts, seeded_image
from posfeat_amd import _lib
assert _lib.lib().posfeat_ab_build() == 1
bb, hd = seeded_state_dicts(0)
imgs = torch.from_numpy(np.stack([seeded_image(s, %(h)d, %(w)d) for s in %(seeds)r])).cuda()
out = {}
for tag, env in (("ref", {}), ("alt", %(env)r)):
    os.environ.update(env)
    eng = ExtractionEngine(bb, hd, device="cuda:0")
    eng.run(imgs)
    r = eng.run(imgs)
    for k in ("local_point", "local_map", "global_feat"):
        out[tag + "_" + k] = r[k].cpu().numpy()
    eng.close()
np.savez(%(out)r, **out)
"""


def _ab_pair(tmp_path, env, H, W, seeds):
    """(default, switched) outputs from one child process on the A/B build."""
    from conftest import ab_env
    out = str(tmp_path / "ab_pair.npz")
    code = AB_CHILD % dict(root=ROOT, h=H, w=W, seeds=tuple(seeds), env=env, out=out)
    subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **ab_env()), check=True,
                   timeout=240)
    d = np.load(out)
    keys = ("local_point", "local_map", "global_feat")
    return ({k: torch.from_numpy(d["ref_" + k]) for k in keys},
            {k: torch.from_numpy(d["alt_" + k]) for k in keys})


def _oracle(img_cpu):
    from oracle import model_ref
    from posfeat_amd.weights import seeded_state_dicts
    bb, hd = seeded_state_dicts(0)
    torch.set_num_threads(min(16, os.cpu_count() or 4))
    return model_ref.posfeat_extract(bb, hd, img_cpu)


def _check_kp_sets(S_ref, got, ref, r, thr, delta):
    from near_tie import explain_differences
    unexplained, overlap = explain_differences(S_ref, got, ref, r, thr, delta)
    assert unexplained.size == 0, "differences not explained by near-ties: %s" % unexplained[:10]
    return overlap


@pytest.mark.parametrize("B", [8, 32])
def test_bench_instance_matches_b1_and_oracle(gpu, B):
    """The B-image 480x640 instance the bench times (B = 32, its default, and
    the round-1 B = 8), after its autotuning forward."""
    from posfeat_amd import ops
    from posfeat_amd.weights import seeded_image
    H, W = 480, 640
    engB = _new_engine(gpu)
    imgs = torch.from_numpy(np.stack([seeded_image(i, H, W) for i in range(B)])).to(gpu)
    engB.run(imgs)                       # first forward: autotune (serial)
    outB = engB.run(imgs)                # the configuration the bench times (side stream)
    lpB = outB["local_point"].clone()
    lmB = outB["local_map"].clone()
    idxB, coordB, scoreB, _, nB = ops.detect(lpB, 1, 2048, thr=0.9, thr_mod="abs")
    descB = ops.sample_desc_nhwc(outB["_local_map_nhwc"], coordB, c=128)
    assert nB == 2048
    eng1 = _new_engine(gpu)
    for i in range(B):
        o1 = eng1.run(imgs[i:i + 1])
        lp1 = o1["local_point"]
        tol.check("local_point", lpB[i:i + 1], lp1, "B%d image %d vs B1" % (B, i))
        tol.check("local_map", lmB[i:i + 1], o1["local_map"], "B%d image %d vs B1" % (B, i))
        idx1, coord1, score1, _, n1 = ops.detect(lp1, 1, 2048, thr=0.9, thr_mod="abs")
        gotB, got1 = idxB[i].cpu().numpy(), idx1[0].cpu().numpy()
        if not np.array_equal(gotB, got1):
            delta = float((lpB[i] - lp1[0]).abs().max())
            ov = _check_kp_sets(lp1[0, 0].cpu().numpy(), gotB, got1, 1, 0.9, delta)
            assert ov > 0.97
        else:
            d1 = ops.sample_desc_nhwc(o1["_local_map_nhwc"], coord1, c=128)
            e, _ = _maxerr(descB[i], d1[0])
            assert e <= TOL, "image %d descriptors err %g" % (i, e)
    # two of the images against the torch-CPU oracle
    for i in (0, B - 3):
        ref = _oracle(imgs[i:i + 1].cpu())
        tol.check("local_point", lpB[i:i + 1], ref["local_point"], "B%d image %d vs oracle" % (B, i))
        tol.check("local_map", lmB[i:i + 1], ref["local_map"], "B%d image %d vs oracle" % (B, i))
    eng1.close()
    engB.close()


@pytest.mark.parametrize("hw", [(768, 1024), (496, 656)])
def test_aachen_shapes_vs_oracle(gpu, hw):
    """Non-480x640 shapes end to end (engine + detector r=3 / thr 0.5 + sampler)."""
    from oracle import detect_ref
    from posfeat_amd import ops
    from posfeat_amd.weights import seeded_image
    H, W = hw
    img = torch.from_numpy(seeded_image(11, H, W))[None]
    eng = _new_engine(gpu)
    out = eng.run(img.to(gpu))
    out = eng.run(img.to(gpu))
    ref = _oracle(img)
    for k in ("local_point", "local_map", "global_map", "global_feat"):
        tol.check(k, out[k], ref[k], "%dx%d vs oracle" % hw)
    S_ref = ref["local_point"][0, 0].numpy()
    lp = out["local_point"]
    delta = float(np.abs(lp[0, 0].cpu().numpy() - S_ref).max())
    cfg = dict(nms_radius=3, num_pts=20480, thr=0.5, thr_mod="abs")
    idx, coord, score, _, n = ops.detect(lp, cfg["nms_radius"], cfg["num_pts"], thr=cfg["thr"],
                                         thr_mod="abs")
    c_ref, s_ref, i_ref = detect_ref.generate_kpts_single(S_ref[None, None], cfg["nms_radius"],
                                                          cfg["num_pts"], thr=cfg["thr"],
                                                          thr_mod="abs", return_idx=True)
    got = idx[0].cpu().numpy()
    if not np.array_equal(got, i_ref[0]):
        ov = _check_kp_sets(S_ref, got, i_ref[0], cfg["nms_radius"], cfg["thr"], delta)
        assert ov > 0.97
    common, ia, ib = np.intersect1d(got, i_ref[0], return_indices=True)
    np.testing.assert_allclose(coord[0].cpu().numpy()[ia], c_ref[0][ib], atol=TOL)
    np.testing.assert_allclose(score[0, :, 0].cpu().numpy()[ia], s_ref[0, :, 0][ib], atol=TOL)
    desc = ops.sample_desc_nhwc(out["_local_map_nhwc"], coord, c=128)[0].cpu().numpy()
    d_ref = detect_ref.sample_feat_by_coord(ref["local_map"].numpy(), c_ref, True)[0]
    np.testing.assert_allclose(desc[ia], d_ref[ib], atol=TOL)
    # the detector on the reference's own map is bit-exact
    idx2, _, _, _, _ = ops.detect(torch.from_numpy(S_ref)[None, None].to(gpu), cfg["nms_radius"],
                                  cfg["num_pts"], thr=cfg["thr"], thr_mod="abs")
    np.testing.assert_array_equal(idx2[0].cpu().numpy(), i_ref[0])
    eng.close()


@pytest.mark.parametrize("switch,exact", [("POSFEAT_SIDE", True), ("POSFEAT_UP4WINO", False),
                                          ("POSFEAT_UP4TAP", False), ("POSFEAT_IMGSTATS", False),
                                          ("POSFEAT_DISK_FLASH", True)])
def test_env_switch_paths_match_default(gpu, switch, exact, tmp_path):
    env = {switch: "0"}
    if switch == "POSFEAT_UP4WINO":
        env["POSFEAT_UP4TAP"] = "0"   # the phase kernel sits behind both
    ref, got = _ab_pair(tmp_path, env, 96, 128, (4, 5))
    for k in ("local_point", "local_map", "global_feat"):
        if exact:
            assert torch.equal(got[k], ref[k]), "%s=0 changed %s" % (switch, k)
        else:
            tol.check(k, got[k], ref[k], "%s=0 vs default" % switch)


@pytest.mark.parametrize("B,hw", [(2, (96, 128)), (2, (112, 144)), (1, (112, 144))])
def test_fused_head_matches_unfused(gpu, B, hw, tmp_path):
    """POSFEAT_HEADFUSE: head.conv2's G part inside the tap combine
    (up4tap_gcombine_kernel, the default) against the G pass + combine
    (gfuse_conv5_k80_kernel + up4tap_combine_kernel): the same products, so
    local_point within 1e-4 absolute -- including a ragged last column
    block (W = 144: 16 of the block's 32 columns), the border ring and both
    block orders (the XCD remap applies when the grid is a multiple of 8:
    B = 2 here; B = 1 at 112 x 144 is 140 blocks)."""
    H, W = hw
    seeds = tuple(range(3, 3 + B))
    ab_ref, got = _ab_pair(tmp_path, {"POSFEAT_HEADFUSE": "0"}, H, W, seeds)
    tol.check("local_point", got["local_point"], ab_ref["local_point"], "HEADFUSE=0 vs default")
    assert torch.equal(got["local_map"], ab_ref["local_map"])   # the backbone is untouched
    # the shipped library's fused head (this process) against the A/B build's
    # default path and the oracle
    from posfeat_amd.weights import seeded_image
    imgs = torch.from_numpy(np.stack([seeded_image(s, H, W) for s in seeds])).to(gpu)
    base = _new_engine(gpu)
    base.run(imgs)
    ref = {k: v.clone() for k, v in base.run(imgs).items() if not k.startswith("_")}
    base.close()
    assert torch.equal(ref["local_point"].cpu(), ab_ref["local_point"])
    o = _oracle(imgs[:1].cpu())
    tol.check("local_point", ref["local_point"][:1], o["local_point"], "fused head vs oracle")


def test_engine_weight_cache_and_weights_changed(gpu):
    """Extraction instances build their derived weights (the blob's bf16
    planes, the decoder's Winograd-domain weights) once, in their own memory:
    repeated runs -- interleaved with another shape's instance on the shared
    workspace -- equal a fresh engine's; after an in-place weight change,
    weights_changed() makes the next run equal a fresh engine built on the
    changed blob."""
    from posfeat_amd.weights import seeded_image
    imgs = torch.from_numpy(np.stack([seeded_image(s, 96, 128) for s in (7, 8)])).to(gpu)
    other = torch.from_numpy(np.stack([seeded_image(9, 64, 96)])).to(gpu)
    eng = _new_engine(gpu)
    first = {k: v.clone() for k, v in eng.run(imgs).items() if not k.startswith("_")}
    eng.run(other)          # another instance writes the shared workspace
    again = eng.run(imgs)
    for k in ("local_point", "local_map", "global_feat"):
        assert torch.equal(again[k], first[k]), k
    # rewrite a decoder conv's weights in place (a Winograd layer) and the head
    spec = {n: (w_off, cout * kpad) for n, cout, cin, kh, kw, kpad, w_off, b_off in
            _specs_with_kpad()}
    for name in ("upconv2.conv", "iconv2", "head.conv1"):
        off, n = spec[name]
        eng.wdev[off:off + n] *= 1.25
    eng.weights_changed()
    got = eng.run(imgs)
    fresh = _new_engine(gpu)
    fresh.wdev.copy_(eng.wdev)
    ref = fresh.run(imgs)
    for k in ("local_point", "local_map", "global_feat"):
        assert torch.equal(got[k], ref[k]), k
    for k in ("local_point", "local_map"):   # global_feat does not see these layers
        assert not torch.equal(got[k], first[k]), k
    eng.close()
    fresh.close()


def _specs_with_kpad():
    from posfeat_amd import _lib, weights
    out = []
    for name, cout, cin, kh, kw, w_off, b_off in _lib.model_specs():
        out.append((name, cout, cin, kh, kw, weights.packed_k(cin, kh, kw)[2], w_off, b_off))
    return out


def test_engine_shape_cache_lru_and_shared_workspace(gpu, monkeypatch):
    """Many image sizes (HPatches / Aachen): at most POSFEAT_ENGINE_MAX_SHAPES
    instances are kept (least recently used evicted), inference instances
    share one grow-only workspace, and a shape planned after an eviction (its
    tiles from the process-wide cache, or from a similar shape) gives the
    same maps as a fresh engine."""
    from posfeat_amd.weights import seeded_image
    monkeypatch.setenv("POSFEAT_ENGINE_MAX_SHAPES", "2")
    eng = _new_engine(gpu)
    shapes = [(96, 128), (128, 160), (112, 144), (96, 128)]
    outs = []
    for h, w in shapes:
        img = torch.from_numpy(seeded_image(7, h, w))[None].to(gpu)
        o = eng.run(img)
        outs.append({k: o[k].clone() for k in ("local_point", "local_map")})
        assert len(eng.cached_shapes) <= 2
    assert eng.cached_shapes == [(1, 112, 144), (1, 96, 128)]
    assert eng.workspace_bytes == eng._shared_ws.numel()
    for k in ("local_point", "local_map"):          # re-planned shape: same result
        assert torch.equal(outs[0][k], outs[3][k]), k
    fresh = _new_engine(gpu)
    img = torch.from_numpy(seeded_image(7, 112, 144))[None].to(gpu)
    ref = fresh.run(img)
    for k in ("local_point", "local_map"):
        tol.check(k, outs[2][k], ref[k], "re-planned shape vs fresh")
    fresh.close()
    eng.close()
