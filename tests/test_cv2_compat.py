"""cv2-shaped shims and the Matching-shaped callable.

CPU part: host Rodrigues vs the oracle's restatement of cv2.Rodrigues, unsupported
parameters are refused, and calls fail loudly without a GPU.  GPU part: the reference's
own lines (stereo_slam.py:232-238, :262, :294-306 and :210-218) run through the shims and
give the oracle's keypoints, descriptors, matches, disparities and pose."""
import numpy as np
import pytest
import torch

from conftest import gpu_available


def _cv2():
    from forest_slam_amd import cv2_compat
    return cv2_compat


# ----------------------------------------------------------------------------- CPU
def test_rodrigues_vector_matches_oracle(oracle_mod):
    cv2 = _cv2()
    rng = np.random.default_rng(0)
    vecs = [np.zeros(3), np.array([1e-20, 0, 0]), np.array([0, 0, np.pi]), np.array([0.3, -0.2, 0.1])]
    vecs += list(rng.normal(0, 1.0, (20, 3)))
    for r in vecs:
        R, J = cv2.Rodrigues(r.reshape(3, 1))
        Ro, Jo = oracle_mod.rodrigues_jac(r)
        np.testing.assert_allclose(R, Ro, rtol=0, atol=1e-15)
        np.testing.assert_allclose(J, Jo, rtol=0, atol=1e-14)


def test_rodrigues_matrix_roundtrip_matches_oracle(oracle_mod):
    cv2 = _cv2()
    rng = np.random.default_rng(1)
    for r in list(rng.normal(0, 0.8, (20, 3))) + [np.zeros(3), np.array([0, np.pi, 0]), np.array([np.pi, 0, 0])]:
        R, _ = cv2.Rodrigues(r)
        back, _ = cv2.Rodrigues(R)
        np.testing.assert_allclose(back.reshape(3), oracle_mod.rodrigues_inv(R), rtol=0, atol=1e-10)


def test_unsupported_parameters_are_refused():
    cv2 = _cv2()
    with pytest.raises(NotImplementedError):
        cv2.ORB_create(WTA_K=3)
    with pytest.raises(NotImplementedError):
        cv2.ORB_create(scoreType=1)
    with pytest.raises(NotImplementedError):
        cv2.BFMatcher(cv2.NORM_HAMMING, crossCheck=False)
    with pytest.raises(NotImplementedError):
        cv2.StereoSGBM_create(numDisparities=96, blockSize=7, mode=cv2.STEREO_SGBM_MODE_SGBM)
    with pytest.raises(NotImplementedError):
        cv2.StereoSGBM_create(numDisparities=96, blockSize=5, mode=cv2.STEREO_SGBM_MODE_SGBM_3WAY)
    with pytest.raises(NotImplementedError):
        cv2.solvePnPRansac(np.zeros((8, 3)), np.zeros((8, 2)), np.eye(3), None, useExtrinsicGuess=True)
    with pytest.raises(NotImplementedError):
        cv2.findEssentialMat(np.zeros((8, 2)), np.zeros((8, 2)), focal=500.0, pp=(0, 0), method=4)
    with pytest.raises(NotImplementedError):
        cv2.findEssentialMat(np.zeros((8, 2)), np.zeros((8, 2)), np.diag([500.0, 501.0, 1.0]))
    with pytest.raises(NotImplementedError):
        cv2.recoverPose(np.eye(3), np.zeros((8, 2)), np.zeros((8, 2)), focal=500.0, mask=np.ones((8, 1), np.uint8))


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure path")
def test_shims_fail_loudly_without_gpu():
    cv2 = _cv2()
    with pytest.raises(RuntimeError):
        cv2.ORB_create().detectAndCompute(np.zeros((64, 64), np.uint8), None)
    with pytest.raises(RuntimeError):
        cv2.BFMatcher(cv2.NORM_HAMMING, crossCheck=True).match(np.zeros((4, 32), np.uint8), np.zeros((4, 32), np.uint8))


# ----------------------------------------------------------------------------- GPU
gpu = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]


@pytest.fixture(scope="module")
def seq_frames():
    import forest_slam_amd.synth as synth
    seq = synth.StereoSequence(seed=11, n_frames=3, W=960, H=600, device="cpu")
    return [tuple(x.numpy() for x in seq.frame(i)) for i in range(2)]


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_reference_orb_branch_through_shims(oracle_mod, seq_frames):
    """stereo_slam.py:84-85, :232-238, :108-123, :262-303 verbatim over the shims."""
    cv2 = _cv2()
    from forest_slam_amd import synth
    (prevL, prevR), (curL, _) = seq_frames
    orb = cv2.ORB_create()
    bf_matcher_orb = cv2.BFMatcher(cv2.NORM_HAMMING, crossCheck=True)
    kpts0_l, descs0_l = orb.detectAndCompute(prevL, None)
    kpts1_l, descs1_l = orb.detectAndCompute(curL, None)
    matches_l = bf_matcher_orb.match(descs0_l, descs1_l)
    mkpts0_l = np.float32([kpts.pt for kpts in kpts0_l])
    mkpts1_l = np.float32([kpts.pt for kpts in kpts1_l])
    mkpts0_l = mkpts0_l[[m.queryIdx for m in matches_l]]
    mkpts1_l = mkpts1_l[[m.trainIdx for m in matches_l]]

    ref = oracle_mod.frame_pose(prevL, prevR, curL, synth.K0, synth.DIST_L, synth.BASELINE, nfeatures=500)
    assert np.array_equal(np.float32([k.pt for k in kpts0_l]), ref["kp0"][:, :2])
    assert np.array_equal(descs0_l, ref["d0"]) and np.array_equal(descs1_l, ref["d1"])
    assert np.array_equal(np.array([[m.queryIdx, m.trainIdx, m.distance] for m in matches_l]), ref["matches"])

    matcher = cv2.StereoSGBM_create(numDisparities=6 * 16, minDisparity=0, blockSize=7, P1=8 * 7 ** 2,
                                    P2=32 * 7 ** 2, mode=cv2.STEREO_SGBM_MODE_SGBM_3WAY)
    disp16 = matcher.compute(prevL, prevR)
    assert disp16.dtype == np.int16 and np.array_equal(disp16, ref["disp16"])

    # back-projection exactly as the reference writes it (host NumPy here; the product
    # path is fvo_backproject), then the PnP shim
    disparity_map = disp16.astype(np.float32) / 16
    disparity_map[disparity_map == 0.0] = 0.1
    disparity_map[disparity_map == -1.0] = 0.1
    K0 = synth.K0
    depth = np.float32(K0[0, 0] * synth.BASELINE) / disparity_map
    X, Y = mkpts0_l[:, 0], mkpts0_l[:, 1]
    Z = depth[Y.astype(int), X.astype(int)]
    X = ((X - np.float32(K0[0, 2])) / np.float32(K0[0, 0])) * Z
    Y = ((Y - np.float32(K0[1, 2])) / np.float32(K0[1, 1])) * Z
    points3D = np.column_stack((X, Y, Z))
    valid = (Z > 0.1) & (Z < 1000)
    points3D, mk1 = points3D[valid], mkpts1_l[valid]
    assert np.array_equal(points3D, ref["P3"]) and np.array_equal(mk1, ref["p2"])
    ok, rvec, tvec, inliers = cv2.solvePnPRansac(points3D, mk1, K0, synth.DIST_L, reprojectionError=1.0,
                                                 confidence=0.99, iterationsCount=1000, flags=cv2.SOLVEPNP_ITERATIVE)
    rok, rrv, rtv, rinl = ref["ok"], ref["rvec"], ref["tvec"], ref["inliers"]
    assert ok == rok
    if ok:
        assert np.abs(rvec.reshape(3) - rrv).max() < 1e-4 and np.abs(tvec.reshape(3) - rtv).max() < 1e-4
        assert np.array_equal(inliers.reshape(-1), rinl)
        rotation_mat, _ = cv2.Rodrigues(rvec)
        T = np.eye(4)
        T[:3, :3] = rotation_mat
        T[:3, 3] = tvec.T
        assert np.abs(T - ref["T"]).max() < 1e-4


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_matching_callable_matches_bf_path(oracle_mod, seq_frames):
    """stereo_slam.py:192, :210-218 with ORBMatching in place of SuperGlue's Matching."""
    cv2 = _cv2()
    (prevL, _), (curL, _) = seq_frames
    feature_matcher = cv2.ORBMatching({"nfeatures": 500})
    t0 = torch.from_numpy(prevL / 255.).float()[None, None].cuda()
    t1 = torch.from_numpy(curL / 255.).float()[None, None].cuda()
    pred_left = feature_matcher({'image0': t0, 'image1': t1})
    pred_left = {k: v[0].detach().cpu().numpy() for k, v in pred_left.items()}
    kpts0_l, kpts1_l = pred_left['keypoints0'], pred_left['keypoints1']
    matches_l, conf_l = pred_left['matches0'], pred_left['matching_scores0']
    valid_l = matches_l > -1
    mkpts0_l = kpts0_l[valid_l]
    mkpts1_l = kpts1_l[matches_l[valid_l]]

    kp0, d0 = oracle_mod.orb_detect_compute(prevL, 500)
    kp1, d1 = oracle_mod.orb_detect_compute(curL, 500)
    m = oracle_mod.bf_match(d0, d1)
    assert np.array_equal(mkpts0_l, kp0[m[:, 0], :2]) and np.array_equal(mkpts1_l, kp1[m[:, 1], :2])
    np.testing.assert_array_equal(conf_l[valid_l], (1.0 - m[:, 2] / 256.0).astype(np.float32))
    assert np.all(conf_l[~valid_l] == 0)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_bf_shim_edge_cases(oracle_mod):
    cv2 = _cv2()
    bf = cv2.BFMatcher(cv2.NORM_HAMMING, crossCheck=True)
    rng = np.random.default_rng(5)
    assert bf.match(np.zeros((0, 32), np.uint8), rng.integers(0, 256, (7, 32), dtype=np.uint8)) == []
    with pytest.raises(cv2.error):
        bf.match(None, np.zeros((3, 32), np.uint8))
    # more descriptors than the default capacity: the shim grows its context
    d0 = rng.integers(0, 256, (2500, 32), dtype=np.uint8)
    d1 = rng.integers(0, 256, (1800, 32), dtype=np.uint8)
    got = np.array([[m.queryIdx, m.trainIdx, m.distance] for m in bf.match(d0, d1)])
    assert np.array_equal(got, oracle_mod.bf_match(d0, d1))


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_reference_mono_lines_through_shims(oracle_mod):
    """mono_slam.py:111-117 verbatim over the shims, on ORB+BF matches of two synthetic
    frames, against the oracle."""
    import forest_slam_amd.synth as synth
    cv2 = _cv2()
    seq = synth.StereoSequence(seed=12, n_frames=3, W=960, H=600, device="cpu", start=120)
    I0, I1 = seq.frame(0)[0].numpy(), seq.frame(2)[0].numpy()
    K0 = seq.K
    orb = cv2.ORB_create()
    bf = cv2.BFMatcher(cv2.NORM_HAMMING, crossCheck=True)
    k0, d0 = orb.detectAndCompute(I0, None)
    k1, d1 = orb.detectAndCompute(I1, None)
    matches = bf.match(d0, d1)
    mkpts0 = np.float32([k0[m.queryIdx].pt for m in matches])
    mkpts1 = np.float32([k1[m.trainIdx].pt for m in matches])
    # --- mono_slam.py:111-117
    E, mask = cv2.findEssentialMat(mkpts0, mkpts1, focal=K0[0,0], pp=(K0[0,2], K0[1,2]), method=cv2.RANSAC, prob=0.999, threshold=1.0)
    _, rotation, translation, _ = cv2.recoverPose(E, mkpts0, mkpts1, focal=K0[0,0], pp=(K0[0,2], K0[1,2]))
    translation = translation.reshape(3)
    relative_est_tf_mat = np.eye(4)
    relative_est_tf_mat[:3, 3] = translation
    relative_est_tf_mat[:3, :3] = rotation
    # --- oracle
    st, rE, rmask, _, _ = oracle_mod.find_essential(mkpts0, mkpts1, K0[0, 0], (K0[0, 2], K0[1, 2]))
    assert st == 1
    assert np.abs(E - rE).max() < 1e-9 and np.array_equal(mask.reshape(-1), rmask)
    g, rR, rt = oracle_mod.recover_pose(rE, mkpts0, mkpts1, K0[0, 0], (K0[0, 2], K0[1, 2]))
    assert np.abs(relative_est_tf_mat[:3, :3] - rR).max() < 1e-9
    assert np.abs(relative_est_tf_mat[:3, 3] - rt).max() < 1e-9
