"""Seeded two-view correspondence sets for the mono (essential-matrix) path: a known
relative pose, points in front of both cameras, pixel noise and outliers.  Shared by the
golden generator and the tests (test infrastructure)."""
import numpy as np

F, CX, CY = 642.9165664800531, 460.0, 308.0  # stereo_slam.py:45-47 scale (K0 fx, principal point)


def rot(r):
    th = np.linalg.norm(r)
    if th == 0:
        return np.eye(3)
    k = r / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def two_view(seed, n, noise=0.3, outliers=0.2, forward=True):
    """Returns (p0 f32[n,2], p1 f32[n,2], R, t unit) with x1 ~ R x0 + t."""
    rng = np.random.default_rng(seed)
    R = rot(rng.normal(size=3) * 0.05)
    t = rng.normal(size=3)
    if forward:
        t[2] = abs(t[2]) + 0.5
    t /= np.linalg.norm(t)
    X = np.c_[rng.uniform(-5, 5, n), rng.uniform(-3, 3, n), rng.uniform(4, 30, n)]
    X2 = X @ R.T + t
    p0 = np.c_[F * X[:, 0] / X[:, 2] + CX, F * X[:, 1] / X[:, 2] + CY]
    p1 = np.c_[F * X2[:, 0] / X2[:, 2] + CX, F * X2[:, 1] / X2[:, 2] + CY]
    p1 = p1 + rng.normal(size=p1.shape) * noise
    k = int(round(outliers * n))
    if k:
        p1[rng.choice(n, k, replace=False)] = rng.uniform([0, 0], [920, 616], (k, 2))
    return p0.astype(np.float32), p1.astype(np.float32), R, t


# (seed, n, noise, outliers): edge sizes (no points, too few, exactly 5, 6) and typical sets
CASES = [(1, 0, 0.0, 0.0), (2, 4, 0.0, 0.0), (3, 5, 0.0, 0.0), (4, 6, 0.0, 0.0), (5, 8, 0.2, 0.0),
         (6, 50, 0.3, 0.1), (7, 300, 0.3, 0.2), (8, 300, 0.0, 0.0), (9, 1000, 0.5, 0.4), (10, 120, 1.5, 0.5),
         (11, 2000, 0.3, 0.3)]
