"""Deterministic local-BA problems for the tests (helper module, not a test file).

`clean_problem` builds a stereo VO window with known geometry: landmarks in front of a
forward-moving camera, keypoints = projections + Gaussian noise scaled by a random ORB
octave, one-to-one matches between consecutive frames, stereo disparities with noise,
and relative poses perturbed from the truth (the "PnP" initial guess).  Arrays come in
the frame layout of fvo_ba_windows (keypoint records of 8 floats, match rows, per-keypoint
stereo (X, Y, Z, d)) and in the list layout of oracle/ba_ref.py.
"""
import numpy as np

K_TEST = np.array([[428.6, 0.0, 306.8], [0.0, 428.0, 205.7], [0.0, 0.0, 1.0]])
B_TEST = 0.2537


def _expso3(w):
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * (Kx @ Kx)


def clean_problem(n=10, n_pts=3000, seed=0, W=640, H=400, cap=4096, pose_noise=0.03, drop=0.0):
    rng = np.random.default_rng(seed)
    K, B = K_TEST, B_TEST
    Tg = [np.eye(4)]
    for _ in range(n - 1):
        T = np.eye(4)
        T[:3, :3] = _expso3(rng.normal(0, 0.01, 3))
        T[:3, 3] = [0.01, 0.0, -0.15]
        Tg.append(T @ Tg[-1])
    Tg = np.array(Tg)
    Xw = np.c_[rng.uniform(-8, 8, n_pts), rng.uniform(-3, 2, n_pts), rng.uniform(3, 30, n_pts)]
    kp = np.zeros((n, cap, 8), np.float32)
    nkp = np.zeros(n, np.int32)
    proj = []
    for j in range(n):
        Xc = (Tg[j][:3, :3] @ Xw.T).T + Tg[j][:3, 3]
        u = K[0, 0] * Xc[:, 0] / Xc[:, 2] + K[0, 2]
        v = K[1, 1] * Xc[:, 1] / Xc[:, 2] + K[1, 2]
        vis = (Xc[:, 2] > 0.5) & (u >= 0) & (u < W - 1) & (v >= 0) & (v < H - 1)
        if drop > 0:
            vis &= rng.random(n_pts) >= drop
        idx = np.nonzero(vis)[0][:cap]
        octv = rng.integers(0, 3, len(idx))
        sc = 1.2 ** octv
        kp[j, :len(idx), 0] = u[idx] + rng.normal(0, 0.5, len(idx)) * sc
        kp[j, :len(idx), 1] = v[idx] + rng.normal(0, 0.5, len(idx)) * sc
        kp[j, :len(idx), 5] = octv
        kp[j, :len(idx), 6] = -1
        nkp[j] = len(idx)
        proj.append(idx)
    matches = np.zeros((n, cap, 3), np.int32)
    nmatch = np.zeros(n, np.int32)
    stereo = np.zeros((n, cap, 4), np.float32)
    f32 = np.float32
    for j in range(n - 1):
        pos = {p: i for i, p in enumerate(proj[j + 1])}
        rows = [(i, pos[p], 0) for i, p in enumerate(proj[j]) if p in pos]
        if drop > 0:  # some outlier matches
            rows = [(a, (b + 7) % nkp[j + 1], c) if rng.random() < drop else (a, b, c) for a, b, c in rows]
            seen, uniq = set(), []
            for a, b, c in rows:  # keep the one-to-one property of cross-checked matching
                if b not in seen:
                    seen.add(b)
                    uniq.append((a, b, c))
            rows = uniq
        m = np.array(rows, np.int32).reshape(-1, 3)
        matches[j, :len(m)] = m
        nmatch[j] = len(m)
        Xc = (Tg[j][:3, :3] @ Xw[proj[j]].T).T + Tg[j][:3, 3]
        d = (K[0, 0] * B / Xc[:, 2] + rng.normal(0, 0.3, len(Xc))).astype(f32)
        Z = f32(K[0, 0] * B) / d
        x, y = kp[j, :len(d), 0], kp[j, :len(d), 1]
        X = ((x - f32(K[0, 2])) / f32(K[0, 0])) * Z
        Y = ((y - f32(K[1, 2])) / f32(K[1, 1])) * Z
        ok = (Z > f32(0.1)) & (Z < f32(1000))
        stereo[j, :len(d)] = np.where(ok[:, None], np.stack([X, Y, Z, d], 1), 0).astype(f32)
    relg = np.array([Tg[j + 1] @ np.linalg.inv(Tg[j]) for j in range(n - 1)])
    relp = relg.copy()
    for j in range(n - 1):
        relp[j, :3, 3] += rng.normal(0, pose_noise, 3)
        relp[j, :3, :3] = _expso3(rng.normal(0, pose_noise / 6, 3)) @ relp[j, :3, :3]
    T_rel = np.zeros((n, 4, 4))
    T_rel[:n - 1] = relp
    T_rel[n - 1] = np.eye(4)
    return dict(kp=kp, nkp=nkp, matches=matches, nmatch=nmatch, stereo=stereo, T_rel=T_rel, relg=relg, K=K, B=B)


def oracle_lists(p, s, e):
    """Frames s..e of a frame-layout problem in oracle/ba_ref.py's list layout."""
    kps = [p["kp"][f, :p["nkp"][f], :6] for f in range(s, e + 1)]
    matches = [p["matches"][f, :p["nmatch"][f]] for f in range(s, e)]
    st = []
    for f in range(s, e):
        a = p["stereo"][f, :p["nkp"][f]]
        st.append((a[:, :3], a[:, 3], a[:, 2] > 0))
    return kps, matches, st, p["T_rel"][s:e]
