"""Training-side descriptor correlation -- host side.

Synthetic epipolar geometry for benchmarks and tests (the reference builds F
from MegaDepth poses, datasets/megadepth.py:426-448); the GPU paths for
Preprocess_Line2Window / EpipolarLoss_full / DiskLoss live below.
"""
import numpy as np


def _rotvec(rv):
    th = np.linalg.norm(rv)
    if th < 1e-12:
        return np.eye(3)
    k = rv / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def _skew(x):
    return np.array([[0, -x[2], x[1]], [x[2], 0, -x[0]], [-x[1], x[0], 0]])


def synthetic_fundamental(b, h, w, seed):
    """(F1, F2) float32 [b,3,3]: F = K2^-T [t]x R K1^-1 / F[2,2] for a random
    small relative pose, and its reverse (megadepth.py:426-448, 483-484)."""
    rs = np.random.RandomState(seed)
    f = 0.8 * w
    K = np.array([[f, 0, (w - 1) / 2.0], [0, f, (h - 1) / 2.0], [0, 0, 1.0]])
    Ki = np.linalg.inv(K)
    F1s, F2s = [], []
    for _ in range(b):
        R = _rotvec(rs.normal(0, 0.1, 3))
        t = rs.normal(0, 1, 3)
        t /= np.linalg.norm(t)
        rel = np.eye(4)
        rel[:3, :3], rel[:3, 3] = R, t
        rel2 = np.linalg.inv(rel)
        E1 = _skew(rel[:3, 3]) @ rel[:3, :3]
        E2 = _skew(rel2[:3, 3]) @ rel2[:3, :3]
        F1 = Ki.T @ E1 @ Ki
        F2 = Ki.T @ E2 @ Ki
        F1s.append((F1.astype(np.float32) / np.float32(F1[-1, -1] + 1e-10)).astype(np.float32))
        F2s.append((F2.astype(np.float32) / np.float32(F2[-1, -1] + 1e-10)).astype(np.float32))
    return np.stack(F1s), np.stack(F2s)
