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
