"""Trajectory I/O and accuracy metrics.

* TUM trajectory writer/reader in the reference's layout ``t x y z qx qy qz qw``
  (``stereo_slam.py:337-338,352-360``: ``np.savetxt(..., fmt='%f')``, quaternion from
  ``tf.transformations.quaternion_from_matrix``, xyzw order).
* ATE: evo-equivalent APE on the translation part after Umeyama Sim(3) alignment
  (``evo_ape tum GT EST -as``), nearest-timestamp association within 0.01 s.
  Pinned in tests against the reference's own result files: ORB_BF_Stereo 1018_00 ->
  1.1565 m, and the colour-bar extents of three evo plots (Appendix B).
* RPE: evo-equivalent relative pose error, point-distance error ratio (%) for delta = 20 m
  over consecutive pairs, Sim(3)-aligned (``evo_rpe tum GT EST -as --delta 20 --delta_unit m
  --pose_relation point_distance_error_ratio``) — the metric of the reference's
  ``pose_estimation_results/1018_00/1018-00-{Stereo,Mono}-rpe.png``; pinned in tests against
  the per-pair values and statistics read off those two plots.
"""
from __future__ import annotations

import numpy as np


def quaternion_from_matrix(M: np.ndarray) -> np.ndarray:
    """xyzw quaternion of a 4x4 transform, ROS ``tf.transformations`` semantics
    (trace-based branch selection, no sign normalisation) as used at stereo_slam.py:327."""
    M = np.asarray(M, dtype=np.float64)[:4, :4]
    q = np.empty(4)
    t = np.trace(M)
    if t > M[3, 3]:
        q[3] = t
        q[2] = M[1, 0] - M[0, 1]
        q[1] = M[0, 2] - M[2, 0]
        q[0] = M[2, 1] - M[1, 2]
    else:
        i, j, k = 0, 1, 2
        if M[1, 1] > M[0, 0]:
            i, j, k = 1, 2, 0
        if M[2, 2] > M[i, i]:
            i, j, k = 2, 0, 1
        t = M[i, i] - (M[j, j] + M[k, k]) + M[3, 3]
        q[i] = t
        q[j] = M[i, j] + M[j, i]
        q[k] = M[k, i] + M[i, k]
        q[3] = M[k, j] - M[j, k]
    q *= 0.5 / np.sqrt(t * M[3, 3])
    return q


def tum_rows(stamps, poses) -> np.ndarray:
    rows = []
    for t, T in zip(stamps, poses):
        q = quaternion_from_matrix(T)
        rows.append([t, T[0, 3], T[1, 3], T[2, 3], q[0], q[1], q[2], q[3]])
    return np.array(rows, dtype=np.float64).reshape(-1, 8)


def save_tum(path: str, stamps, poses) -> None:
    np.savetxt(path, tum_rows(stamps, poses), delimiter=" ", fmt="%f")


def load_tum(path: str) -> np.ndarray:
    return np.loadtxt(path, dtype=np.float64).reshape(-1, 8)


def associate(t_ref: np.ndarray, t_est: np.ndarray, max_diff: float = 0.01):
    """Index pairs (i_ref, i_est): nearest reference stamp for every estimate stamp."""
    order = np.argsort(t_ref)
    ts = t_ref[order]
    pos = np.searchsorted(ts, t_est)
    lo = np.clip(pos - 1, 0, len(ts) - 1)
    hi = np.clip(pos, 0, len(ts) - 1)
    pick = np.where(np.abs(ts[hi] - t_est) < np.abs(ts[lo] - t_est), hi, lo)
    ok = np.abs(ts[pick] - t_est) < max_diff
    return order[pick[ok]], np.nonzero(ok)[0]


def umeyama(src: np.ndarray, dst: np.ndarray, with_scale: bool = True):
    """Least-squares s, R, t with dst ~ s R src + t (Umeyama 1991), points as rows."""
    mu_s, mu_d = src.mean(0), dst.mean(0)
    xs, xd = src - mu_s, dst - mu_d
    n = len(src)
    cov = xd.T @ xs / n
    U, D, Vt = np.linalg.svd(cov)
    S = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        S[2, 2] = -1
    R = U @ S @ Vt
    s = (np.trace(np.diag(D) @ S) / ((xs ** 2).sum() / n)) if with_scale else 1.0
    t = mu_d - s * R @ mu_s
    return s, R, t


def ate(ref: np.ndarray, est: np.ndarray, align: str = "sim3", max_diff: float = 0.01) -> dict:
    """APE (translation part) after alignment; ref/est are TUM arrays [N,8]."""
    ir, ie = associate(ref[:, 0], est[:, 0], max_diff)
    P = est[ie, 1:4]
    Q = ref[ir, 1:4]
    if align == "sim3":
        s, R, t = umeyama(P, Q, True)
    elif align == "se3":
        s, R, t = umeyama(P, Q, False)
    else:
        s, R, t = 1.0, np.eye(3), np.zeros(3)
    e = np.linalg.norm((s * (R @ P.T)).T + t - Q, axis=1)
    return dict(rmse=float(np.sqrt(np.mean(e ** 2))), mean=float(e.mean()), median=float(np.median(e)),
                min=float(e.min()), max=float(e.max()), n=int(len(e)), scale=float(s))


def chain(rel: np.ndarray, valid: np.ndarray | None = None) -> np.ndarray:
    """stereo_slam.py:306 ``cumulative = np.dot(cumulative, T)`` left to right, in float64.
    Frames whose pose is invalid (the ``len(points3D) >= 6`` skip, :292) leave the
    cumulative pose unchanged and emit no TUM row (returned mask says which)."""
    cum = np.eye(4)
    out = []
    for i in range(len(rel)):
        if valid is not None and not valid[i]:
            continue
        cum = np.dot(cum, rel[i])
        out.append(cum.copy())
    return np.array(out).reshape(-1, 4, 4)


def path_pairs(positions: np.ndarray, delta: float) -> list[tuple[int, int]]:
    """evo ``filters.filter_pairs_by_path`` (consecutive pairs): walk the trajectory
    accumulating the travelled distance; every index where it reaches ``delta`` (metres) is a
    pair boundary and the counter restarts there.  Pairs join consecutive boundaries (the
    start pose is not a boundary: 4 pairs for the 113.8 m of 1018_00 at delta 20 m)."""
    ids = []
    prev = positions[0]
    acc = 0.0
    for i, p in enumerate(positions):
        acc += float(np.linalg.norm(p - prev))
        prev = p
        if acc >= delta:
            ids.append(i)
            acc = 0.0
    return list(zip(ids, ids[1:]))


def rpe(ref: np.ndarray, est: np.ndarray, delta: float = 20.0, align: str = "sim3", max_diff: float = 0.01,
        pairs_from_reference: bool = False) -> dict:
    """RPE w.r.t. the point-distance error ratio (%), evo semantics: associate (as ``ate``),
    align the estimate (Sim(3) Umeyama by default), pick consecutive pairs (i, j) ``delta``
    metres of path apart on the aligned estimate (evo's default; the reference's with
    ``pairs_from_reference``), and per pair
    ``100 * | |p_ref[j] - p_ref[i]| - |p_est[j] - p_est[i]| | / |p_ref[j] - p_ref[i]|``
    (the norm of the relative SE(3) translation is the position distance).  ``t`` is the
    estimate stamp of each pair's second pose, ``t_rel`` that minus the first stamp."""
    ir, ie = associate(ref[:, 0], est[:, 0], max_diff)
    P = est[ie, 1:4]
    Q = ref[ir, 1:4]
    if align in ("sim3", "se3"):
        s, R, t = umeyama(P, Q, align == "sim3")
        P = (s * (R @ P.T)).T + t
    pairs = path_pairs(Q if pairs_from_reference else P, delta)
    if not pairs:
        return dict(values=np.zeros(0), t=np.zeros(0), t_rel=np.zeros(0), n=0, rmse=float("nan"),
                    mean=float("nan"), median=float("nan"), pairs=[])
    i, j = np.array(pairs).T
    dr = np.linalg.norm(Q[j] - Q[i], axis=1)
    de = np.linalg.norm(P[j] - P[i], axis=1)
    nz = dr > 0
    e = np.abs(dr - de)[nz] / dr[nz] * 100.0
    ts = est[ie, 0]
    return dict(values=e, t=ts[j[nz]], t_rel=ts[j[nz]] - ts[0], n=int(len(e)), rmse=float(np.sqrt(np.mean(e ** 2))),
                mean=float(e.mean()), median=float(np.median(e)), std=float(e.std()), min=float(e.min()),
                max=float(e.max()), pairs=pairs)
