"""Evaluator pins against the reference's own result files (pose_estimation_results/,
copied to tests/golden/) — SURVEY.md §6 and Appendix B."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _load(name):
    from forest_slam_amd import eval as ev
    return ev.load_tum(os.path.join(GOLDEN, name + ".txt"))


@pytest.mark.parametrize("est,rmse", [("1018_00_ORB_BF_Stereo", 1.1565), ("1018_00_ORB_BF_Stereo_K10", 5.8420),
                                      ("1018_00_ORB_BF_Stereo_K20", 11.7265),
                                      ("1018_00_SuperPoint_SuperGlue_Stereo", 0.7770),
                                      ("1018_00_SuperPoint_SuperGlue_Mono", 1.1682)])
def test_ate_sim3_pins(est, rmse):
    from forest_slam_amd import eval as ev
    r = ev.ate(_load("1018_00_Ground_Truth"), _load(est))
    assert abs(r["rmse"] - rmse) < 5e-5


def test_ate_plot_colour_bars():
    """min/max per-pose APE = the colour-bar ends of the reference's evo plots."""
    from forest_slam_amd import eval as ev
    for gt, est, lo, hi in [("1018_00_Ground_Truth", "1018_00_SuperPoint_SuperGlue_Stereo", 0.165, 2.354),
                            ("1018_13_Ground_Truth", "1018_13_SuperPoint_SuperGlue_Stereo", 0.519, 5.775),
                            ("1018_00_Ground_Truth", "1018_00_SuperPoint_SuperGlue_Mono", 0.216, 3.368)]:
        r = ev.ate(_load(gt), _load(est))
        assert round(r["min"], 3) == lo and round(r["max"], 3) == hi


def test_ate_se3_and_scale():
    from forest_slam_amd import eval as ev
    gt, est = _load("1018_00_Ground_Truth"), _load("1018_00_ORB_BF_Stereo")
    assert abs(ev.ate(gt, est, "se3")["rmse"] - 2.5383) < 5e-5
    assert abs(ev.ate(gt, est)["scale"] - 0.880) < 5e-4


def test_quaternion_and_tum_roundtrip(tmp_path):
    from scipy.spatial.transform import Rotation
    from forest_slam_amd import eval as ev
    rng = np.random.default_rng(0)
    poses = []
    for _ in range(20):
        T = np.eye(4)
        T[:3, :3] = Rotation.from_rotvec(rng.normal(0, 1, 3)).as_matrix()
        T[:3, 3] = rng.normal(0, 5, 3)
        poses.append(T)
        q = ev.quaternion_from_matrix(T)
        assert np.allclose(np.abs(q @ Rotation.from_matrix(T[:3, :3]).as_quat()), 1.0, atol=1e-9)
    p = tmp_path / "t.txt"
    ev.save_tum(str(p), np.arange(20) * 0.1, poses)
    back = ev.load_tum(str(p))
    assert back.shape == (20, 8) and np.allclose(back[:, 1:4], np.array(poses)[:, :3, 3], atol=1e-6)


def test_chain_is_left_to_right_and_skips_invalid():
    from forest_slam_amd import eval as ev
    A = np.eye(4); A[:3, 3] = [1, 0, 0]
    Bm = np.eye(4); Bm[:3, :3] = [[0, -1, 0], [1, 0, 0], [0, 0, 1]]
    out = ev.chain(np.stack([A, Bm, A]), np.array([True, False, True]))
    assert out.shape == (2, 4, 4)
    assert np.allclose(out[1], A @ A)
    out = ev.chain(np.stack([A, Bm, A]))
    assert np.allclose(out[2], np.dot(np.dot(A, Bm), A))


# Values read off the reference's evo RPE plots (pose_estimation_results/1018_00/
# 1018-00-Stereo-rpe.png and 1018-00-Mono-rpe.png: "RPE w.r.t. point distance error ratio (%)
# for delta = 20.0 (m) using consecutive pairs (with Sim(3) Umeyama alignment)"): per-pair
# (seconds from start, RPE %) vertices of the grey curve and the rmse / mean / median lines.
# The plot reading resolution is ~0.05 % and ~0.3 s.
RPE_PLOTS = {
    "1018_00_SuperPoint_SuperGlue_Stereo": dict(
        t=[35.5, 49.8, 65.2, 79.3], v=[4.62, 0.37, 0.51, 1.14], rmse=2.40, mean=1.65, median=0.82),
    "1018_00_SuperPoint_SuperGlue_Mono": dict(
        t=[29.8, 44.7, 59.6, 74.5, 89.4], v=[6.85, 2.80, 6.03, 5.82, 0.35], rmse=5.00, mean=4.36, median=5.82),
}


@pytest.mark.parametrize("est", sorted(RPE_PLOTS))
def test_rpe_matches_reference_plots(est):
    """evo RPE restatement (eval.rpe) reproduces the reference's two RPE plots: the pair
    count, each pair's time and error ratio, and the summary lines."""
    from forest_slam_amd import eval as ev
    want = RPE_PLOTS[est]
    r = ev.rpe(_load("1018_00_Ground_Truth"), _load(est), delta=20.0)
    assert r["n"] == len(want["v"])
    assert np.allclose(r["t_rel"], want["t"], atol=0.35)
    assert np.allclose(r["values"], want["v"], atol=0.06)
    for k in ("rmse", "mean", "median"):
        assert abs(r[k] - want[k]) < 0.06, (k, r[k])


def test_rpe_orb_bf_stereo_and_properties():
    """The ORB+BF stereo result (the reference CPU path; no RPE plot is published for it):
    4 pairs over the 113.8 m path; identical trajectories give 0 %; a pure scale error of the
    estimate is removed by the Sim(3) alignment but not by the SE(3) one."""
    from forest_slam_amd import eval as ev
    gt, est = _load("1018_00_Ground_Truth"), _load("1018_00_ORB_BF_Stereo")
    r = ev.rpe(gt, est)
    assert r["n"] == 4 and 3.9 < r["mean"] < 4.1
    assert ev.rpe(gt, gt)["rmse"] < 1e-9
    scaled = gt.copy()
    scaled[:, 1:4] *= 0.5
    assert ev.rpe(gt, scaled)["rmse"] < 1e-6
    assert abs(ev.rpe(gt, scaled, align="se3")["mean"] - 50.0) < 1e-6
