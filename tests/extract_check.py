"""Near-tie-aware check of extract.py output files against the oracle.

An ``.npz`` holds refined keypoint positions (pixels), scores and descriptors,
not the selected pixel indices.  Each keypoint is mapped back to its pixel by
the oracle's soft-argmax refinement map (oracle/detect_ref.refine_maps): the
file's position of pixel p is the GPU's refinement of p, which differs from the
oracle's by the map difference (~1e-5), while distinct pixels' refinements are
~1/W apart.  The selected index sets must then differ only where the deciding
comparison is a near-tie in the oracle's map (tests/near_tie.py, with
``delta`` = max |S_gpu - S_ref| of an in-process GPU run with the same batch
composition), and at every common pixel position / score / descriptor agree
within 1e-4.
"""
import numpy as np

from near_tie import explain_differences

MATCH_TOL = 1e-3   # normalised units (0.08 px at w = 160)


def file_indices(kpt_px, rx, ry, h, w):
    """Inner-pixel index of each file keypoint (refinement within MATCH_TOL)."""
    cx, cy = (w - 1) / 2.0, (h - 1) / 2.0
    nx = (kpt_px[:, 0].astype(np.float64) - cx) / cx
    ny = (kpt_px[:, 1].astype(np.float64) - cy) / cy
    hi, wi = rx.shape
    out = np.empty(len(kpt_px), np.int64)
    for k in range(len(kpt_px)):
        # full-res pixel nearest the position, as an inner index, +-2 around it
        ci = int(round(float(kpt_px[k, 1]))) - 1
        cj = int(round(float(kpt_px[k, 0]))) - 1
        best, bi = np.inf, -1
        for i in range(max(0, ci - 2), min(hi, ci + 3)):
            for j in range(max(0, cj - 2), min(wi, cj + 3)):
                d = max(abs(rx[i, j] - nx[k]), abs(ry[i, j] - ny[k]))
                if d < best:
                    best, bi = d, i * wi + j
        assert best <= MATCH_TOL, "keypoint %d (%s) matches no pixel's refinement (%.2e)" % (
            k, kpt_px[k], best)
        out[k] = bi
    return out


def check_file(z, ref, S_ref, delta, det_cfg, h, w, tag=""):
    """z: the loaded npz; ref: detect_ref.process_image output for the image;
    S_ref: oracle score map (h, w); delta: max |S_gpu - S_ref|."""
    from oracle.detect_ref import refine_maps
    kp, sc, de = z["keypoints"], z["scores"], z["descriptors"]
    assert kp.dtype == np.float32 and sc.dtype == np.float32 and de.dtype == np.float32, tag
    assert kp.ndim == 2 and kp.shape[1] == 2 and sc.shape == (len(kp), 1), tag
    assert de.shape == (len(kp), 128), tag
    np.testing.assert_allclose(np.linalg.norm(de, axis=1), 1.0, atol=1e-5, err_msg=tag)
    rx, ry = refine_maps(S_ref)
    got = file_indices(kp, rx, ry, h, w)
    assert len(set(got.tolist())) == len(got), "%s: two keypoints on one pixel" % tag
    want = ref["idx"][0]
    assert len(got) == len(want), "%s: %d keypoints, oracle %d" % (tag, len(got), len(want))
    r = det_cfg.get("nms_radius", 1)
    thr = det_cfg.get("thr", None) if det_cfg.get("thr_mod", "abs") == "abs" else None
    # Filler entries: when the image has fewer NMS/threshold survivors than n
    # (n is raised to 128, or n = num_pts > count), top-k pads with entries of
    # masked score 0, which the reference's torch.topk orders arbitrarily:
    # they are compared by count only.  An entry outside the
    # oracle's mask is a filler unless its deciding comparison is a near-tie
    # (then it is a survivor in the GPU map and explain_differences judges it).
    from near_tie import _margins
    from oracle.detect_ref import _mask_and_inner
    _, mask = _mask_and_inner(S_ref[None, None], r, True, det_cfg.get("thr", False),
                              det_cfg.get("thr_mod", "mean"))
    mask = mask[0].reshape(-1)
    marg = _margins(S_ref, r, thr, None)

    def survivors(idx):
        return np.array([p for p in idx if mask[p] or marg[p] <= 2 * delta + 1e-7], np.int64)
    got_s, want_s = survivors(got), survivors(want)
    unexplained, overlap = explain_differences(S_ref, got_s, want_s, r, thr, delta)
    assert unexplained.size == 0, "%s: %d selection differences not explained by near-ties " \
        "(delta %.2e): %s" % (tag, unexplained.size, delta, unexplained[:8])
    pos = {int(p): i for i, p in enumerate(want) if mask[p]}
    a = np.array([i for i, p in enumerate(got) if int(p) in pos], np.int64)
    b = np.array([pos[int(got[i])] for i in a], np.int64)
    assert len(a) >= 1, tag
    pxtol = 1e-4 * max(w - 1, h - 1) / 2.0   # 1e-4 in normalised coordinates
    np.testing.assert_allclose(kp[a], ref["kpt"][b], atol=pxtol, rtol=0, err_msg=tag)
    np.testing.assert_allclose(sc[a], ref["kp_score"][0][b], atol=1e-4, err_msg=tag)
    np.testing.assert_allclose(de[a], ref["desc"][0][b], atol=1e-4, err_msg=tag)
    return overlap, len(kp), len(want)
