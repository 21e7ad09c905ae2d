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


# ----------------------------------------------------------------------- motion-blur ablation
# apply_random_motion_blur (forest_slam_ros/src/stereo_slam.py:142-178).
# Parity vs OpenCV is unpinned (no cv2 here): the oracle restates filter2D's direct float path
# (k*k < 130) and the exact S/k of its DFT path (k*k >= 130); both are checked below against
# an independent integer evaluation away from exact ties.

def _blur_numpy(img, k, centers):
    """Independent restatement: exact S/k rounded (ties reported), the reference's mask loop."""
    H, W = img.shape
    a = k // 2
    p = np.pad(img.astype(np.int64), k, mode="reflect")  # numpy 'reflect' == BORDER_REFLECT_101
    S = sum(p[k - a + i:k - a + i + H, k - a + i:k - a + i + W] for i in range(k))
    mask = np.zeros((H, W), np.uint8)
    for pix in centers:  # stereo_slam.py:167-171
        y, x = pix // W, pix % W
        mask[max(0, y - a):min(H, y + a + 1), max(0, x - a):min(W, x + a + 1)] = 1
    return np.floor(S / k + 0.5), (S % k) * 2 == k, mask


def test_golden_blur_reproduces(oracle_mod):
    g = np.load(os.path.join(GOLDEN, "golden_blur.npz"))
    for k in (10, 15, 20):
        out, mask = oracle_mod.motion_blur(g["img"], k, g["centers"])
        assert np.array_equal(out, g[f"out{k}"]) and np.array_equal(mask, g[f"mask{k}"])


@pytest.mark.parametrize("k", [3, 10, 11, 12, 15, 20])
def test_blur_oracle_matches_exact_sum(oracle_mod, k):
    rng = np.random.default_rng(k)
    img = rng.integers(0, 256, (48, 70), dtype=np.uint8)
    centers = rng.choice(48 * 70, 40, replace=False).astype(np.int32)
    out, mask = oracle_mod.motion_blur(img, k, centers)
    exact, tie, mask_np = _blur_numpy(img, k, centers)
    assert np.array_equal(mask, mask_np)
    assert np.array_equal(out[mask == 0], img[mask == 0])
    sel = (mask == 1) & ~tie
    assert np.array_equal(out[sel], exact[sel].astype(np.uint8))
    if k * k >= 130:  # DFT path: ties half to even
        q = np.floor(exact - 0.5)
        want = np.where(q % 2 == 0, q, q + 1)
        assert np.array_equal(out[(mask == 1) & tie], want[(mask == 1) & tie].astype(np.uint8))


def test_blur_zero_percent_is_identity(oracle_mod):
    # the reference's active call: blur_percentage=0, kernel_size=20 (stereo_slam.py:194, :206)
    from forest_slam_amd.cv2_compat import blur_centers
    img = np.random.default_rng(2).integers(0, 256, (40, 64), dtype=np.uint8)
    c = blur_centers(40, 64, 0)
    assert c.size == 0
    out, mask = oracle_mod.motion_blur(img, 20, c)
    assert np.array_equal(out, img) and mask.sum() == 0


def test_blur_centers_follow_random_sample():
    import random
    from forest_slam_amd.cv2_compat import blur_centers
    c = blur_centers(600, 960, 10, random.Random(3))
    assert c.dtype == np.int32 and len(c) == int(600 * 960 * 0.1)
    assert np.array_equal(c, random.Random(3).sample(range(600 * 960), len(c)))


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_gpu_motion_blur_matches_oracle(oracle_mod):
    import random
    from forest_slam_amd import _lib
    for (W, H) in [(960, 600), (333, 211)]:
        ctx = _lib.Context(W, H, max_batch=3, stages=_lib.STAGE_BF, kp_capacity=64)
        imgs = np.stack([synthetic_bgr(H, W, s)[..., 1] for s in range(3)])
        imgs[2] = np.random.default_rng(9).integers(0, 256, (H, W), dtype=np.uint8)
        t = torch.from_numpy(imgs).cuda()
        for k, pct in [(10, 1), (15, 0.5), (20, 10), (20, 0), (3, 2)]:
            cs = [np.asarray(random.Random(b + k).sample(range(H * W), int(H * W * pct / 100)), np.int32)
                  for b in range(3)]
            cap = max(1, max(len(c) for c in cs))
            C = np.zeros((3, cap), np.int32)
            for b, c in enumerate(cs):
                C[b, :len(c)] = c
            n = torch.tensor([len(c) for c in cs], dtype=torch.int32, device="cuda")
            out, mask = ctx.motion_blur(t, k, torch.from_numpy(C).cuda(), n)
            out, mask = out.cpu().numpy(), mask.cpu().numpy()
            for b in range(3):
                want, wmask = oracle_mod.motion_blur(imgs[b], k, cs[b])
                assert np.array_equal(mask[b], wmask), (W, H, k, b)
                assert np.array_equal(out[b], want), (W, H, k, b, int((out[b] != want).sum()))


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_gpu_apply_random_motion_blur_shim(oracle_mod):
    import random
    from forest_slam_amd import cv2_compat as cv2
    img = synthetic_bgr(600, 960, 4)[..., 0].copy()
    got = cv2.apply_random_motion_blur(img, blur_percentage=10, kernel_size=15, rng=random.Random(1))
    want, _ = oracle_mod.motion_blur(img, 15, cv2.blur_centers(600, 960, 10, random.Random(1)))
    assert np.array_equal(got, want)
    # the reference's active call (:194): 0 % blurred -> the image itself
    assert np.array_equal(cv2.apply_random_motion_blur(img, blur_percentage=0, kernel_size=20, angle=0), img)
    with pytest.raises(NotImplementedError):
        cv2.apply_random_motion_blur(img, 10, 15, angle=30)
