"""ORACLE — test infrastructure only (the specification of the windowed local BA).

Local bundle adjustment over a sliding window of K frames (SURVEY.md §8 a15,
BASELINE.json north_star "local BA").  The reference has no BA (it chains PnP poses,
stereo_slam.py:306), so there is nothing upstream to pin: this float64 NumPy restatement
IS the definition the HIP kernel (forest-slam_amd/csrc/ba.hip) is checked against —
parity unpinned with respect to the reference by construction.  Only tests/ may import it.

Window ending at frame e: frames s..e (n = e - s + 1 <= K), world = camera s.
  * poses: T_j (world -> camera j), T_s = I fixed; initialised by composing the front
    end's relative transforms (camera j -> camera j+1, the PnP output).
  * landmarks: for j = s..e-1 and each BF match row (q, t) of L_j -> L_{j+1} in row
    order, keypoint q starts a landmark when it is not the train keypoint of a match
    L_{j-1} -> L_j inside the window (j > s) and its stereo depth is valid (the
    reference's back-projection, float32: d = disp16/16 with 0 / -1 -> 0.1,
    Z = fx*B/d, 0.1 < Z < 1000).  Its track follows the match chain to frame e.
    Creation stops at the first landmark that would exceed LMAX landmarks or OMAX obs.
  * observations: (u, v) in every tracked frame, plus the right-image column
    uR = u - d in the first frame (a stereo observation, which fixes the scale).
  * residual: pinhole projection (images are undistorted before ORB) minus measurement,
    weighted by the keypoint's pyramid level: s = |r|^2 / sigma2[octave] with
    sigma2[o] = scale_factor ** (2 o) (ORB keypoints of level o are quantised o-fold
    coarser); Huber on s with delta^2 = 5.991 (mono) / 7.815
    (stereo): rho(s) = s (s <= d2) else 2 sqrt(d2 s) - d2, IRLS weight rho'(s);
    observations with camera depth <= 0.01 are ignored.  cost = sum rho / 2.
  * Levenberg-Marquardt: H + lam*diag(H) + 1e-6 I, lam0 = 1e-3, /10 on accept (>= 1e-7),
    *10 on reject (<= 1e7); `iters` linearisations.  Before linearisation iters // 2
    (iters >= 2) the observations with s > delta^2 or camera depth <= 0.01 at the current
    estimate are dropped for the rest of the solve (weight 0, the ORB-SLAM local-BA
    schedule) and the current cost is re-evaluated.  Pose update left-multiplicative on
    SO(3) x R3: R <- Exp(w) R, t <- Exp(w) t + v; landmarks X <- X + dX.
  * solve: landmarks eliminated (Schur complement), reduced pose system by Cholesky.
"""
from __future__ import annotations

import numpy as np

LMAX = 4096
OMAX = 32768
D2_MONO = 5.991
D2_STEREO = 7.815
LAM0 = 1e-3
MIN_Z = 0.01


def stereo_points(kp_xy: np.ndarray, disp16: np.ndarray, K: np.ndarray, baseline: float):
    """Per keypoint of a left image: (X_cam f32[n,3], disparity f32[n], valid bool[n]),
    the float32 back-projection of stereo_slam.py:265-289 (NumPy 1.x rules)."""
    f32 = np.float32
    x = kp_xy[:, 0].astype(f32)
    y = kp_xy[:, 1].astype(f32)
    d = disp16[y.astype(int), x.astype(int)].astype(f32) / f32(16)
    d[d == f32(0.0)] = f32(0.1)
    d[d == f32(-1.0)] = f32(0.1)
    Z = f32(K[0, 0] * baseline) / d
    X = ((x - f32(K[0, 2])) / f32(K[0, 0])) * Z
    Y = ((y - f32(K[1, 2])) / f32(K[1, 1])) * Z
    valid = (Z > f32(0.1)) & (Z < f32(1000))
    return np.stack([X, Y, Z], 1).astype(f32), d, valid


def build_problem(kps, matches, stereo, rel, lmax=LMAX, omax=OMAX, scale_factor=1.2):
    """kps: n frames of f32[n_f, >=6] keypoint records (x, y, size, angle, response,
    octave, ...); matches: n-1 int[M, 3] (L_j -> L_{j+1});
    stereo: n-1 (P f32[n_j,3], d f32[n_j], valid) for the frames with forward matches;
    rel: f64[n-1, 4, 4] camera j -> camera j+1.  Returns (T0 f64[n,4,4], X f64[L,3],
    obs dict of arrays lm, frame, u, v, ur (nan = mono), isig2 (1 / sigma2[octave]))."""
    n = len(kps)
    T = np.zeros((n, 4, 4))
    T[0] = np.eye(4)
    for j in range(n - 1):
        T[j + 1] = rel[j] @ T[j]
    nxt = []
    for j in range(n - 1):
        a = np.full(len(kps[j]), -1, np.int64)
        m = np.asarray(matches[j]).reshape(-1, 3)
        a[m[:, 0]] = m[:, 1]
        nxt.append(a)
    X, o_lm, o_f, o_u, o_v, o_ur, o_is = [], [], [], [], [], [], []
    stop = False
    for j in range(n - 1):
        tracked = np.zeros(len(kps[j]), bool)
        if j > 0:
            tracked[np.asarray(matches[j - 1]).reshape(-1, 3)[:, 1]] = True
        P, d, valid = stereo[j]
        Tinv = np.linalg.inv(T[j])
        for q, t, _ in np.asarray(matches[j]).reshape(-1, 3):
            if tracked[q] or not valid[q]:
                continue
            chain = [(j, q), (j + 1, t)]
            f, b = j + 1, t
            while f < n - 1 and nxt[f][b] >= 0:
                b = nxt[f][b]
                f += 1
                chain.append((f, b))
            if len(X) + 1 > lmax or len(o_lm) + len(chain) > omax:
                stop = True
                break
            lm = len(X)
            Xc = P[q].astype(np.float64)
            X.append(Tinv[:3, :3] @ Xc + Tinv[:3, 3])
            for k, (ff, kk) in enumerate(chain):
                o_lm.append(lm)
                o_f.append(ff)
                o_u.append(float(kps[ff][kk, 0]))
                o_v.append(float(kps[ff][kk, 1]))
                o_ur.append(float(np.float32(kps[j][q, 0]) - d[q]) if k == 0 else np.nan)
                o_is.append(1.0 / (scale_factor ** (2 * int(kps[ff][kk, 5]))))
        if stop:
            break
    obs = dict(lm=np.array(o_lm, np.int64), frame=np.array(o_f, np.int64), u=np.array(o_u),
               v=np.array(o_v), ur=np.array(o_ur), isig2=np.array(o_is))
    return T, np.array(X).reshape(-1, 3), obs


def _expso3(w):
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * (Kx @ Kx)


def _linearize(T, X, obs, cam, baseline, need_jac=True):
    fx, fy, cx, cy = cam
    R = T[obs["frame"], :3, :3]
    t = T[obs["frame"], :3, 3]
    Xc = np.einsum("nij,nj->ni", R, X[obs["lm"]]) + t
    x, y, z = Xc[:, 0], Xc[:, 1], Xc[:, 2]
    ok = z > MIN_Z
    zs = np.where(ok, z, 1.0)
    iz = 1.0 / zs
    st = ~np.isnan(obs["ur"])
    r = np.zeros((len(z), 3))
    r[:, 0] = fx * x * iz + cx - obs["u"]
    r[:, 1] = fy * y * iz + cy - obs["v"]
    r[:, 2] = np.where(st, fx * (x - baseline) * iz + cx - np.nan_to_num(obs["ur"]), 0.0)
    s = (r ** 2).sum(1) * obs["isig2"]
    d2 = np.where(st, D2_STEREO, D2_MONO)
    inl = s <= d2
    rho = np.where(inl, s, 2.0 * np.sqrt(d2 * s) - d2)
    w = np.where(inl, 1.0, np.sqrt(d2 / np.maximum(s, 1e-300)))
    rho = np.where(ok, rho, 0.0)
    w = np.where(ok, w * obs["isig2"], 0.0)  # IRLS weight x information
    cost = 0.5 * rho.sum()
    if not need_jac:
        return cost
    # d(proj)/d(Xc): rows u, v, uR
    Jc = np.zeros((len(z), 3, 3))
    Jc[:, 0, 0] = fx * iz
    Jc[:, 0, 2] = -fx * x * iz * iz
    Jc[:, 1, 1] = fy * iz
    Jc[:, 1, 2] = -fy * y * iz * iz
    Jc[:, 2, 0] = np.where(st, fx * iz, 0.0)
    Jc[:, 2, 2] = np.where(st, -fx * (x - baseline) * iz * iz, 0.0)
    # d(Xc)/d(w, v) = [-[Xc]x, I]; d(Xc)/dX = R
    skew = np.zeros((len(z), 3, 6))
    skew[:, 0, 1], skew[:, 0, 2] = z, -y
    skew[:, 1, 0], skew[:, 1, 2] = -z, x
    skew[:, 2, 0], skew[:, 2, 1] = y, -x
    skew[:, 0, 3] = skew[:, 1, 4] = skew[:, 2, 5] = 1.0
    Jp = np.einsum("nij,njk->nik", Jc, skew)
    Jl = np.einsum("nij,njk->nik", Jc, R)
    return cost, r, w, Jp, Jl


def _reject(T, X, obs, cam, baseline):
    """Drop (weight 0) the observations that are outliers at the current estimate."""
    fx, fy, cx, cy = cam
    R = T[obs["frame"], :3, :3]
    t = T[obs["frame"], :3, 3]
    Xc = np.einsum("nij,nj->ni", R, X[obs["lm"]]) + t
    x, y, z = Xc[:, 0], Xc[:, 1], Xc[:, 2]
    ok = z > MIN_Z
    iz = 1.0 / np.where(ok, z, 1.0)
    st = ~np.isnan(obs["ur"])
    r0 = fx * x * iz + cx - obs["u"]
    r1 = fy * y * iz + cy - obs["v"]
    r2 = np.where(st, fx * (x - baseline) * iz + cx - np.nan_to_num(obs["ur"]), 0.0)
    s = (r0 * r0 + r1 * r1 + r2 * r2) * obs["isig2"]
    keep = ok & (s <= np.where(st, D2_STEREO, D2_MONO))
    out = dict(obs)
    out["isig2"] = np.where(keep, obs["isig2"], 0.0)
    return out


def _solve(T, X, obs, lin, lam, n):
    cost, r, w, Jp, Jl = lin
    L = len(X)
    Hpp = np.zeros((n, 6, 6))
    gp = np.zeros((n, 6))
    Hll = np.zeros((L, 3, 3))
    gl = np.zeros((L, 3))
    Wb = np.einsum("nki,n,nkj->nij", Jp, w, Jl)  # 6x3 per obs
    np.add.at(Hpp, obs["frame"], np.einsum("nki,n,nkj->nij", Jp, w, Jp))
    np.add.at(gp, obs["frame"], np.einsum("nki,n,nk->ni", Jp, w, r))
    np.add.at(Hll, obs["lm"], np.einsum("nki,n,nkj->nij", Jl, w, Jl))
    np.add.at(gl, obs["lm"], np.einsum("nki,n,nk->ni", Jl, w, r))
    eye3, eye6 = np.eye(3), np.eye(6)
    Hll_d = Hll + lam * Hll * eye3 + 1e-6 * eye3
    Hpp_d = Hpp + lam * Hpp * eye6 + 1e-6 * eye6
    Hll_inv = np.linalg.inv(Hll_d)
    npz = 6 * (n - 1)
    S = np.zeros((npz, npz))
    rhs = np.zeros(npz)
    for j in range(1, n):
        S[6 * (j - 1):6 * j, 6 * (j - 1):6 * j] = Hpp_d[j]
        rhs[6 * (j - 1):6 * j] = -gp[j]
    # Schur complement: S -= sum_l W_l Hll^-1 W_l^T ; rhs += W_l Hll^-1 g_l
    for l in range(L):
        idx = np.nonzero(obs["lm"] == l)[0]
        fr = obs["frame"][idx]
        keep = fr > 0
        idx, fr = idx[keep], fr[keep]
        Hi = Hll_inv[l]
        for a, fa in zip(idx, fr):
            WaHi = Wb[a] @ Hi
            rhs[6 * (fa - 1):6 * fa] += WaHi @ gl[l]
            for b, fb in zip(idx, fr):
                S[6 * (fa - 1):6 * fa, 6 * (fb - 1):6 * fb] -= WaHi @ Wb[b].T
    try:
        Lc = np.linalg.cholesky(S)
    except np.linalg.LinAlgError:
        return None
    dp = np.linalg.solve(Lc.T, np.linalg.solve(Lc, rhs))
    dpf = np.zeros((n, 6))
    dpf[1:] = dp.reshape(n - 1, 6)
    # back-substitution: dX_l = Hll^-1 (-g_l - sum_obs W^T dp_frame)
    b = -gl.copy()
    np.add.at(b, obs["lm"], -np.einsum("nij,ni->nj", Wb, dpf[obs["frame"]]))
    dX = np.einsum("lij,lj->li", Hll_inv, b)
    return dpf, dX


def _apply(T, X, dpf, dX):
    T2 = T.copy()
    for j in range(1, len(T)):
        Rw = _expso3(dpf[j, :3])
        T2[j, :3, :3] = Rw @ T[j, :3, :3]
        T2[j, :3, 3] = Rw @ T[j, :3, 3] + dpf[j, 3:]
    return T2, X + dX


def ba_window(kps, matches, stereo, rel, K, baseline, iters=10, lmax=LMAX, omax=OMAX, scale_factor=1.2):
    """Windowed LM bundle adjustment (module docstring).  Returns dict with refined poses
    T f64[n,4,4] (world = first camera), rel f64[n-1,4,4] refined relative transforms,
    X f64[L,3], obs, cost0, cost, accepted (number of accepted steps)."""
    T, X, obs = build_problem(kps, matches, stereo, rel, lmax, omax, scale_factor)
    n = len(kps)
    cam = (float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2]))
    lam = LAM0
    cost0 = cost = _linearize(T, X, obs, cam, baseline, need_jac=False) if len(X) else 0.0
    accepted = 0
    for it in range(iters if len(X) else 0):
        if it == iters // 2 and iters >= 2:
            obs = _reject(T, X, obs, cam, baseline)
            cost = _linearize(T, X, obs, cam, baseline, need_jac=False)
        lin = _linearize(T, X, obs, cam, baseline)
        step = _solve(T, X, obs, lin, lam, n)
        if step is None:
            lam = min(lam * 10, 1e7)
            continue
        T2, X2 = _apply(T, X, *step)
        c2 = _linearize(T2, X2, obs, cam, baseline, need_jac=False)
        if c2 < cost:
            T, X, cost = T2, X2, c2
            lam = max(lam / 10, 1e-7)
            accepted += 1
        else:
            lam = min(lam * 10, 1e7)
    relr = np.array([T[j + 1] @ np.linalg.inv(T[j]) for j in range(n - 1)]).reshape(-1, 4, 4)
    return dict(T=T, rel=relr, X=X, obs=obs, cost0=cost0, cost=cost, accepted=accepted)
