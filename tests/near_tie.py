"""Near-tie-aware comparison of two keypoint selections.

NMS / threshold / top-k decisions are discontinuous: if the GPU score map
differs from the reference map by at most ``delta`` everywhere, a decision can
only flip where the deciding comparison has margin <= 2*delta in the
reference map.  ``explain_differences`` returns the indices in the symmetric
difference of the two selections that are NOT explained that way (must be
empty for parity)."""
import numpy as np


def _margins(S, r, thr, cut):
    """Per inner pixel: smallest |difference| among the comparisons that decide
    its selection (window neighbours, threshold, top-k cut)."""
    inner = S[1:-1, 1:-1].astype(np.float64)
    h, w = inner.shape
    p = np.pad(inner, r, mode="reflect")
    m = np.full(inner.shape, np.inf)
    for dy in range(2 * r + 1):
        for dx in range(2 * r + 1):
            if dy == r and dx == r:
                continue
            m = np.minimum(m, np.abs(p[dy:dy + h, dx:dx + w] - inner))
    if thr is not None:
        m = np.minimum(m, np.abs(inner - thr))
    if cut is not None:
        m = np.minimum(m, np.abs(inner - cut))
    return m.reshape(-1)


def explain_differences(S_ref, idx_a, idx_b, r, thr, delta):
    a, b = set(map(int, idx_a)), set(map(int, idx_b))
    diff = np.array(sorted(a ^ b), dtype=np.int64)
    if diff.size == 0:
        return diff, 1.0
    inner = S_ref[1:-1, 1:-1].reshape(-1)
    cut = float(min(inner[np.array(sorted(a), dtype=np.int64)]))
    marg = _margins(S_ref, r, thr, cut)
    unexplained = diff[marg[diff] > 2 * delta + 1e-7]
    return unexplained, len(a & b) / max(1, len(a))
