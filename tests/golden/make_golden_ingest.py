"""Generate tests/golden/golden_ingest.npz with the oracle: cv2.undistort + BGR2GRAY
(stereo_slam.py:184-186) of a seeded synthetic BGR image with the reference's left-camera
intrinsics and distortion (stereo_slam.py:45-50) scaled to 320x200.  No reference fixture
exists for this path; the vector pins the oracle against regressions.
    python tests/golden/make_golden_ingest.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import oracle  # noqa: E402

K0 = np.array([[642.9165664800531, 0., 460.1840658156501], [0., 641.9171825800378, 308.5846449100310], [0., 0., 1.]])
DIST_L = np.array([-0.060164620903866, 0.094005180631043, 0.0, 0.0, 0])


def synthetic_bgr(H, W, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:H, 0:W].astype(np.float64)
    img = np.empty((H, W, 3), np.uint8)
    for c in range(3):
        f = rng.uniform(0.02, 0.2, 4)
        v = 128 + 60 * np.sin(f[0] * x + f[1] * y) + 40 * np.cos(f[2] * x - f[3] * y) + rng.normal(0, 12, (H, W))
        img[..., c] = np.clip(v, 0, 255).astype(np.uint8)
    return img


def main():
    oracle.build()
    W, H = 320, 200
    K = K0.copy()
    K[0] *= W / 960.0
    K[1] *= H / 600.0
    bgr = synthetic_bgr(H, W, 4)
    gray = oracle.undistort_gray(bgr, K, DIST_L)
    mxy, frac = oracle.undistort_map(H, W, K, DIST_L)
    np.savez_compressed(os.path.join(HERE, "golden_ingest.npz"), bgr=bgr, K=K, dist=DIST_L, gray=gray, mxy=mxy,
                        frac=frac)
    print("golden_ingest.npz", gray.mean())


if __name__ == "__main__":
    main()
