"""Image ingest: cv2.undistort + cvtColor(BGR2GRAY) at
stereo_slam.py:184-186 / :196-198.  CPU: the oracle against its golden vector, the
zero-distortion identity (undistort is a no-op, output = the 14-bit gray conversion) and
the map against an independent float64 evaluation of the distortion model.  GPU: the HIP
kernel bit-exact against the oracle (integer output), including odd widths and pitches."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT, gpu_available

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from make_golden_ingest import DIST_L, K0, synthetic_bgr  # noqa: E402

K1 = np.array([[644.4385505412966, 0., 455.1775919513420], [0., 643.5879520187435, 304.1616226347153], [0., 0., 1.]])
DIST_R = np.array([-0.057705696896734, 0.086955444511364, 0.0, 0.0, 0])


def _gray(bgr):
    b, g, r = (bgr[..., k].astype(np.int64) for k in range(3))
    return ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)


def test_golden_ingest_reproduces(oracle_mod):
    g = np.load(os.path.join(GOLDEN, "golden_ingest.npz"))
    assert np.array_equal(oracle_mod.undistort_gray(g["bgr"], g["K"], g["dist"]), g["gray"])
    mxy, fr = oracle_mod.undistort_map(200, 320, g["K"], g["dist"])
    assert np.array_equal(mxy, g["mxy"]) and np.array_equal(fr, g["frac"])


def test_zero_distortion_is_gray_conversion(oracle_mod):
    bgr = synthetic_bgr(120, 200, 1)
    K = K0.copy()
    K[0] *= 200 / 960
    K[1] *= 120 / 600
    assert np.array_equal(oracle_mod.undistort_gray(bgr, K, np.zeros(5)), _gray(bgr))


def test_map_matches_distortion_model(oracle_mod):
    H, W = 600, 960
    mxy, fr = oracle_mod.undistort_map(H, W, K0, DIST_L)
    u_o = mxy[..., 0] + (fr & 31) / 32.0
    v_o = mxy[..., 1] + (fr >> 5) / 32.0
    y, x = np.mgrid[0:H, 0:W].astype(np.float64)
    xn, yn = (x - K0[0, 2]) / K0[0, 0], (y - K0[1, 2]) / K0[1, 1]
    r2 = xn * xn + yn * yn
    kr = 1 + (DIST_L[1] * r2 + DIST_L[0]) * r2
    u = K0[0, 0] * xn * kr + K0[0, 2]
    v = K0[1, 1] * yn * kr + K0[1, 2]
    assert np.abs(u_o - u).max() <= 1 / 64 + 1e-9 and np.abs(v_o - v).max() <= 1 / 64 + 1e-9


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_gpu_undistort_gray_matches_oracle(oracle_mod):
    from forest_slam_amd import _lib
    for (W, H), cams in [((960, 600), [(K0, DIST_L), (K1, DIST_R)]), ((333, 211), [(K0 * [[333 / 960], [211 / 600], [1]], DIST_L)]),
                         ((320, 200), [(K0 * [[1 / 3], [1 / 3], [1]], np.zeros(5))])]:
        ctx = _lib.Context(W, H, max_batch=3, stages=_lib.STAGE_ORB)
        imgs = np.stack([synthetic_bgr(H, W, s) for s in range(3)])
        imgs[2] = np.random.default_rng(9).integers(0, 256, (H, W, 3), dtype=np.uint8)
        t = torch.from_numpy(imgs).cuda()
        for K, d in cams:
            K = np.asarray(K, np.float64)
            got = ctx.undistort_gray(t, K, d).cpu().numpy()
            for b in range(3):
                want = oracle_mod.undistort_gray(imgs[b], K, d)
                assert np.array_equal(got[b], want), (W, H, b, int((got[b] != want).sum()))
