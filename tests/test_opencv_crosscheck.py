"""Guarded cross-check of the oracle against the real libraries the reference calls
("if the GPU box happens to have cv2 … a one-off cross-check cv2 vs cpu_ref on
the fixtures would upgrade the 'unpinned' status; guarded with try: import cv2").  Neither
OpenCV nor Open3D is installed in this image, so these tests skip here and on the GPU box;
wherever they are importable they pin the restatement stage by stage on synthetic frames
(the reference's own inputs, the BotanicGarden bags, are not available)."""
import os
import random
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from make_golden_ingest import DIST_L, K0, synthetic_bgr  # noqa: E402


def _frames():
    from forest_slam_amd import synth
    seq = synth.StereoSequence(seed=3, n_frames=2, W=320, H=200, device="cpu")
    return [tuple(x.numpy() for x in seq.frame(i)) for i in range(2)], seq.K


def test_orb_bf_sgbm_match_opencv(oracle_mod):
    cv2 = pytest.importorskip("cv2")
    (f0, f1), K = _frames()
    orb = cv2.ORB_create(nfeatures=500)  # stereo_slam.py:84
    bf = cv2.BFMatcher(cv2.NORM_HAMMING, crossCheck=True)
    kp_cv, d_cv = orb.detectAndCompute(f0[0], None)
    kp, d = oracle_mod.orb_detect_compute(f0[0], 500)
    assert len(kp_cv) == len(kp)
    assert np.array_equal(np.array([k.pt for k in kp_cv], np.float32), kp[:, :2].astype(np.float32))
    assert np.array_equal(d_cv, d)
    kp1_cv, d1_cv = orb.detectAndCompute(f1[0], None)
    m_cv = bf.match(d_cv, d1_cv)
    _, d1 = oracle_mod.orb_detect_compute(f1[0], 500)
    m = oracle_mod.bf_match(d, d1)
    assert np.array_equal(np.array([(x.queryIdx, x.trainIdx, int(x.distance)) for x in m_cv]).reshape(-1, 3), m)
    sg = cv2.StereoSGBM_create(numDisparities=64, minDisparity=0, blockSize=7, P1=392, P2=1568,
                               mode=cv2.STEREO_SGBM_MODE_SGBM_3WAY)
    assert np.array_equal(sg.compute(f0[0], f0[1]), oracle_mod.sgbm(f0[0], f0[1], num_disp=64))


def test_ingest_and_motion_blur_match_opencv(oracle_mod):
    cv2 = pytest.importorskip("cv2")
    bgr = synthetic_bgr(200, 320, 2)
    K = K0 * [[1 / 3], [1 / 3], [1]]
    want = cv2.cvtColor(cv2.undistort(bgr, K, DIST_L), cv2.COLOR_BGR2GRAY)  # stereo_slam.py:184-186
    assert np.array_equal(oracle_mod.undistort_gray(bgr, K, DIST_L), want)
    gray = want
    for k in (10, 15):  # the reference's apply_motion_blur (forest_slam_ros/src/stereo_slam.py:142-154)
        M = cv2.getRotationMatrix2D((k // 2, k // 2), 0, 1)
        kern = cv2.warpAffine(np.diag(np.ones(k)), M, (k, k)) / k
        blurred = cv2.filter2D(gray, -1, kern)
        centers = np.asarray(random.Random(k).sample(range(200 * 320), 200 * 320 // 10), np.int32)
        out, mask = oracle_mod.motion_blur(gray, k, centers)
        assert np.array_equal(out[mask == 1], blurred[mask == 1])


def test_voxel_down_sample_matches_open3d(oracle_mod):
    o3d = pytest.importorskip("open3d")
    P = np.random.default_rng(0).standard_normal((5000, 3)) * 4
    pcd = o3d.geometry.PointCloud()
    pcd.points = o3d.utility.Vector3dVector(P)
    got = np.asarray(pcd.voxel_down_sample(voxel_size=0.5).points)  # mono_slam.py:155
    want = oracle_mod.voxel_down_sample(P, 0.5)
    assert np.array_equal(got[np.lexsort(got.T[::-1])], want[np.lexsort(want.T[::-1])])
