"""ORACLE — test infrastructure only.

ctypes front-end to ``liboracle.so`` (the scalar C++ restatement of the reference's
OpenCV calls, see ``orb_ref.cpp``, ``bf_ref.cpp``, ``sgbm_ref.cpp``, ``pnp_ref.cpp``).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / CPU baseline — never as the product.

Reference call sites restated here (all in ``ros_ws/src/stereo_slam.py``):
  :84,232-233,240-241  ORB_create() / detectAndCompute        -> orb_detect_compute
  :85,234,242          BFMatcher(NORM_HAMMING, True).match    -> bf_match
  :108-123             StereoSGBM 3-way compute + 0/-1 -> 0.1  -> sgbm / disparity_map
  :265-289             depth, back-projection, 0.1<Z<1000      -> backproject
  :294-306             solvePnPRansac + Rodrigues + chain      -> solve_pnp_ransac / frame_pose
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# FVO_ORACLE_LIB: the sanitizer build (oracle/Makefile.asan, tools/sanitize.sh)
_LIB = os.environ.get("FVO_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")
_lib = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_i16p = ctypes.POINTER(ctypes.c_int16)
_i32p = ctypes.POINTER(ctypes.c_int32)
_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)


def build(force: bool = False) -> str:
    """Compile liboracle.so with the committed Makefile (host g++ only)."""
    if force or not os.path.exists(_LIB):
        subprocess.check_call(["make", "-s", "-C", _HERE] + (["-B"] if force else []))
    return _LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        L.ref_orb_detect_compute.restype = ctypes.c_int
        L.ref_orb_pyramid.restype = ctypes.c_int
        L.ref_fast_detect.restype = ctypes.c_int
        L.ref_retain_best.restype = ctypes.c_int
        L.ref_fast_atan2.restype = ctypes.c_float
        L.ref_fast_atan2.argtypes = [ctypes.c_float, ctypes.c_float]
        L.ref_bf_match.restype = ctypes.c_int
        L.ref_solve_pnp_ransac.restype = ctypes.c_int
        L.ref_find_essential.restype = ctypes.c_int
        L.ref_find_essential.argtypes = [_f32p, _f32p, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                         ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int, _f64p,
                                         _u8p, _i32p, _i32p]
        L.ref_recover_pose.restype = ctypes.c_int
        L.ref_recover_pose.argtypes = [_f64p, _f32p, _f32p, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_double, _f64p, _f64p]
        L.ref_five_point.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


# ----------------------------------------------------------------------------- ORB
def orb_detect_compute(img: np.ndarray, nfeatures: int = 500, fast_threshold: int = 20):
    """Returns (kp f32[N,6] = x,y,size,angle,response,octave, desc u8[N,32])."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    H, W = img.shape
    cap = max(4 * nfeatures, 64)
    while True:
        kp = np.zeros((cap, 6), np.float32)
        desc = np.zeros((cap, 32), np.uint8)
        n = lib().ref_orb_detect_compute(_p(img, _u8p), H, W, W, nfeatures, fast_threshold,
                                         _p(kp, _f32p), _p(desc, _u8p), cap)
        if n >= 0:
            return kp[:n].copy(), desc[:n].copy()
        cap = -n


def orb_pyramid(img: np.ndarray, nlevels: int = 8, blurred: bool = False):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    H, W = img.shape
    sizes = np.zeros((nlevels, 2), np.int32)
    total = lib().ref_orb_pyramid(_p(img, _u8p), H, W, W, nlevels, None, _p(sizes, _i32p), int(blurred))
    buf = np.zeros(total, np.uint8)
    lib().ref_orb_pyramid(_p(img, _u8p), H, W, W, nlevels, _p(buf, _u8p), _p(sizes, _i32p), int(blurred))
    out, off = [], 0
    for w, h in sizes:
        out.append(buf[off:off + w * h].reshape(h, w))
        off += w * h
    return out


def fast_score_map(img: np.ndarray, threshold: int = 20) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    H, W = img.shape
    out = np.zeros((H, W), np.uint8)
    lib().ref_fast_score_map(_p(img, _u8p), H, W, W, threshold, _p(out, _u8p))
    return out


def fast_detect(img: np.ndarray, threshold: int = 20) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    H, W = img.shape
    cap = 1 << 16
    while True:
        out = np.zeros((cap, 3), np.int32)
        n = lib().ref_fast_detect(_p(img, _u8p), H, W, W, threshold, _p(out, _i32p), cap)
        if n >= 0:
            return out[:n].copy()
        cap = -n


def retain_best(resp: np.ndarray, keep: int) -> np.ndarray:
    resp = np.ascontiguousarray(resp, dtype=np.float32)
    out = np.zeros(len(resp), np.int32)
    n = lib().ref_retain_best(_p(resp, _f32p), len(resp), keep, _p(out, _i32p))
    return out[:n].copy()


def fast_atan2(y: float, x: float) -> float:
    return lib().ref_fast_atan2(y, x)


def features_per_level(nfeatures: int = 500, nlevels: int = 8) -> np.ndarray:
    out = np.zeros(nlevels, np.int32)
    lib().ref_features_per_level(nfeatures, nlevels, _p(out, _i32p))
    return out


# ----------------------------------------------------------------------------- BF
def bf_match(d0: np.ndarray, d1: np.ndarray):
    """Returns int32[M,3] rows (queryIdx, trainIdx, distance), ascending queryIdx."""
    d0 = np.ascontiguousarray(d0, dtype=np.uint8)
    d1 = np.ascontiguousarray(d1, dtype=np.uint8)
    n = min(len(d0), len(d1))
    q = np.zeros(max(n, 1), np.int32)
    t = np.zeros(max(n, 1), np.int32)
    d = np.zeros(max(n, 1), np.int32)
    m = lib().ref_bf_match(_p(d0, _u8p), len(d0), _p(d1, _u8p), len(d1), _p(q, _i32p), _p(t, _i32p), _p(d, _i32p))
    return np.stack([q[:m], t[:m], d[:m]], 1)


# ----------------------------------------------------------------------------- SGBM
def sgbm(L: np.ndarray, R: np.ndarray, num_disp: int = 96, block: int = 7, P1: int = 392, P2: int = 1568,
         min_disp: int = 0, raw: bool = False):
    L = np.ascontiguousarray(L, dtype=np.uint8)
    R = np.ascontiguousarray(R, dtype=np.uint8)
    H, W = L.shape
    out = np.zeros((H, W), np.int16)
    rawo = np.zeros((H, W), np.int16)
    lib().ref_sgbm(_p(L, _u8p), _p(R, _u8p), H, W, W, min_disp, num_disp, block, P1, P2, _p(out, _i16p),
                   _p(rawo, _i16p))
    return (out, rawo) if raw else out


def sgbm_row_cost(L, R, y, num_disp=96):
    L = np.ascontiguousarray(L, dtype=np.uint8)
    R = np.ascontiguousarray(R, dtype=np.uint8)
    H, W = L.shape
    width1 = W - num_disp
    out = np.zeros((width1, num_disp), np.int16)
    lib().ref_sgbm_row_cost(_p(L, _u8p), _p(R, _u8p), H, W, W, y, num_disp, _p(out, _i16p))
    return out


def disparity_map(disp16: np.ndarray) -> np.ndarray:
    """stereo_slam.py:117-121: /16 in float32, 0.0 and -1.0 -> 0.1 (float32)."""
    return disparity_map_np1(disp16)


# ----------------------------------------------------------------------------- pose
def backproject(disp_f32: np.ndarray, mk0: np.ndarray, mk1: np.ndarray, K: np.ndarray, baseline: float):
    """stereo_slam.py:265-289 with the reference environment's NumPy 1.x promotion rules
    (Ubuntu 20.04 / Python 3.8: NumPy <= 1.24, value-based casting): a float64 *scalar*
    combined with a float32 *array* computes in float32.  So depth, X, Y, Z and points3D
    are float32; the float64 scalars are rounded to float32 first.  This container runs
    NumPy 2, hence the explicit casts."""
    f32 = np.float32
    cx, cy, fx, fy = K[0, 2], K[1, 2], K[0, 0], K[1, 1]
    depth = f32(fx * baseline) / disp_f32.astype(f32)
    X = mk0[:, 0].astype(f32)
    Y = mk0[:, 1].astype(f32)
    Z = depth[Y.astype(int), X.astype(int)]
    X = ((X - f32(cx)) / f32(fx)) * Z
    Y = ((Y - f32(cy)) / f32(fy)) * Z
    P = np.column_stack((X, Y, Z)).astype(f32)
    valid = (Z > f32(0.1)) & (Z < f32(1000))
    return P[valid], mk1[valid], valid


def disparity_map_np1(disp16: np.ndarray) -> np.ndarray:
    """stereo_slam.py:117-121 (float32 throughout under NumPy 1.x)."""
    d = disp16.astype(np.float32) / np.float32(16)
    d[d == np.float32(0.0)] = np.float32(0.1)
    d[d == np.float32(-1.0)] = np.float32(0.1)
    return d


def solve_pnp_ransac(P3: np.ndarray, p2: np.ndarray, K: np.ndarray, dist: np.ndarray, reproj: float = 1.0,
                     confidence: float = 0.99, iters: int = 1000):
    """Returns (ok, rvec, tvec, inlier_idx, ransac_iters, ransac_inliers)."""
    P3 = np.ascontiguousarray(P3, dtype=np.float64)
    p2 = np.ascontiguousarray(p2, dtype=np.float32)
    K = np.ascontiguousarray(K, dtype=np.float64)
    dist = np.ascontiguousarray(np.resize(np.asarray(dist, np.float64), 5))
    n = len(P3)
    rv = np.zeros(3)
    tv = np.zeros(3)
    mask = np.zeros(max(n, 1), np.uint8)
    ni = np.zeros(1, np.int32)
    bg = np.zeros(1, np.int32)
    ok = lib().ref_solve_pnp_ransac(_p(P3, _f64p), _p(p2, _f32p), n, _p(K, _f64p), _p(dist, _f64p), iters,
                                    ctypes.c_float(reproj), ctypes.c_double(confidence), _p(rv, _f64p),
                                    _p(tv, _f64p), _p(mask, _u8p), _p(ni, _i32p), _p(bg, _i32p))
    return bool(ok), rv, tv, np.nonzero(mask[:n])[0].astype(np.int32), int(ni[0]), int(bg[0])


def find_essential(p1: np.ndarray, p2: np.ndarray, focal: float, pp, prob: float = 0.999, threshold: float = 1.0,
                   max_iters: int = 1000):
    """cv2.findEssentialMat(p1, p2, focal=, pp=, RANSAC, prob, threshold) (mono_slam.py:111).
    Returns (status, E 3x3, inlier mask u8[n], ransac_iters, ransac_inliers); status 1 ok,
    0 RANSAC failed, -1 fewer than 5 points, -2 five points with several solutions."""
    p1 = np.ascontiguousarray(p1, dtype=np.float32).reshape(-1, 2)
    p2 = np.ascontiguousarray(p2, dtype=np.float32).reshape(-1, 2)
    n = len(p1)
    E = np.zeros(9)
    mask = np.zeros(max(n, 1), np.uint8)
    ni = np.zeros(1, np.int32)
    bg = np.zeros(1, np.int32)
    st = lib().ref_find_essential(_p(p1, _f32p), _p(p2, _f32p), n, focal, float(pp[0]), float(pp[1]), prob,
                                  threshold, max_iters, _p(E, _f64p), _p(mask, _u8p), _p(ni, _i32p), _p(bg, _i32p))
    return int(st), E.reshape(3, 3), mask[:n], int(ni[0]), int(bg[0])


def recover_pose(E: np.ndarray, p1: np.ndarray, p2: np.ndarray, focal: float, pp, dist: float = 50.0):
    """cv2.recoverPose(E, p1, p2, focal=, pp=) (mono_slam.py:112) -> (good, R 3x3, t 3)."""
    E = np.ascontiguousarray(E, dtype=np.float64).reshape(9)
    p1 = np.ascontiguousarray(p1, dtype=np.float32).reshape(-1, 2)
    p2 = np.ascontiguousarray(p2, dtype=np.float32).reshape(-1, 2)
    R = np.zeros(9)
    t = np.zeros(3)
    g = lib().ref_recover_pose(_p(E, _f64p), _p(p1, _f32p), _p(p2, _f32p), len(p1), focal, float(pp[0]),
                               float(pp[1]), dist, _p(R, _f64p), _p(t, _f64p))
    return int(g), R.reshape(3, 3), t


def five_point(x1: np.ndarray, x2: np.ndarray) -> np.ndarray:
    """EMEstimatorCallback::runKernel on 5 normalised correspondences -> models [k,3,3]."""
    x1 = np.ascontiguousarray(x1, dtype=np.float64).reshape(5, 2)
    x2 = np.ascontiguousarray(x2, dtype=np.float64).reshape(5, 2)
    out = np.zeros(90)
    k = lib().ref_five_point(_p(x1, _f64p), _p(x2, _f64p), _p(out, _f64p))
    return out[:9 * k].reshape(k, 3, 3)


def undistort_gray(bgr: np.ndarray, K: np.ndarray, dist) -> np.ndarray:
    """cv2.cvtColor(cv2.undistort(bgr, K, dist), cv2.COLOR_BGR2GRAY) (stereo_slam.py:184-186)."""
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    H, W = bgr.shape[:2]
    K = np.ascontiguousarray(K, dtype=np.float64).reshape(9)
    d = np.ascontiguousarray(np.resize(np.asarray(dist, np.float64), 5))
    out = np.zeros((H, W), np.uint8)
    lib().ref_undistort_gray(_p(bgr, _u8p), H, W, W * 3, _p(K, _f64p), _p(d, _f64p), _p(out, _u8p))
    return out


def motion_blur(img: np.ndarray, ksize: int, centers) -> tuple:
    """apply_random_motion_blur(img, kernel_size=ksize, angle=0) with the sampled pixels given
    (forest_slam_ros/src/stereo_slam.py:142-178) -> (out u8[H,W], mask u8[H,W])."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    H, W = img.shape
    c = np.ascontiguousarray(centers, dtype=np.int32).reshape(-1)
    out = np.zeros((H, W), np.uint8)
    mask = np.zeros((H, W), np.uint8)
    lib().ref_motion_blur(_p(img, _u8p), H, W, int(ksize), _p(c, _i32p), len(c), _p(mask, _u8p), _p(out, _u8p))
    return out, mask


def map_transform(points: np.ndarray, T: np.ndarray):
    """(cum @ hstack(points, 1).T)[:3].T (stereo_slam.py:308-311) -> (f64 [n,3], float32 PointCloud2 xyz)."""
    P = np.ascontiguousarray(points, dtype=np.float32)
    T = np.ascontiguousarray(T, dtype=np.float64).reshape(16)
    n, st = P.shape
    o64 = np.zeros((n, 3))
    o32 = np.zeros((n, 3), np.float32)
    lib().ref_map_transform(_p(P, _f32p), ctypes.c_int64(n), st, _p(T, _f64p), _p(o64, _f64p), _p(o32, _f32p))
    return o64, o32


def voxel_down_sample(points: np.ndarray, voxel_size: float) -> np.ndarray:
    """Open3D PointCloud.voxel_down_sample (mono_slam.py:155), voxels in (ix, iy, iz) order."""
    P = np.ascontiguousarray(points, dtype=np.float64)
    out = np.zeros((max(len(P), 1), 3))
    lib().ref_voxel_down_sample.restype = ctypes.c_int64
    n = lib().ref_voxel_down_sample(_p(P, _f64p), ctypes.c_int64(len(P)), ctypes.c_double(voxel_size), _p(out, _f64p))
    return out[:n]


def undistort_map(H: int, W: int, K: np.ndarray, dist):
    """(map xy i16[H,W,2], fractional index u16[H,W]) of initUndistortRectifyMap(CV_16SC2)."""
    K = np.ascontiguousarray(K, dtype=np.float64).reshape(9)
    d = np.ascontiguousarray(np.resize(np.asarray(dist, np.float64), 5))
    mxy = np.zeros((H, W, 2), np.int16)
    fr = np.zeros((H, W), np.uint16)
    lib().ref_undistort_map(H, W, _p(K, _f64p), _p(d, _f64p), _p(mxy, _i16p), _p(fr, ctypes.POINTER(ctypes.c_uint16)))
    return mxy, fr


def pnp_hypotheses(P3, p2, K, dist, iters=1000, reproj=1.0):
    """Debug: (models f64[iters,6] (rvec, tvec), inlier counts i32[iters]) of the RANSAC subsets."""
    P3 = np.ascontiguousarray(P3, dtype=np.float64)
    p2 = np.ascontiguousarray(p2, dtype=np.float32)
    K = np.ascontiguousarray(K, dtype=np.float64)
    dist = np.ascontiguousarray(np.resize(np.asarray(dist, np.float64), 5))
    models = np.zeros((iters, 6))
    good = np.zeros(iters, np.int32)
    lib().ref_pnp_hypotheses(_p(P3, _f64p), _p(p2, _f32p), len(P3), _p(K, _f64p), _p(dist, _f64p), iters,
                             ctypes.c_float(reproj), _p(models, _f64p), _p(good, _i32p))
    return models, good


def rodrigues(rvec: np.ndarray) -> np.ndarray:
    rvec = np.ascontiguousarray(rvec, dtype=np.float64).reshape(3)
    R = np.zeros(9)
    lib().ref_rodrigues(_p(rvec, _f64p), _p(R, _f64p))
    return R.reshape(3, 3)


def rodrigues_jac(rvec: np.ndarray):
    """(R 3x3, J 3x9) as cv2.Rodrigues(rvec) returns them."""
    rvec = np.ascontiguousarray(rvec, dtype=np.float64).reshape(3)
    R, J = np.zeros(9), np.zeros(27)
    lib().ref_rodrigues_jac(_p(rvec, _f64p), _p(R, _f64p), _p(J, _f64p))
    return R.reshape(3, 3), J.reshape(3, 9)


def rodrigues_inv(R: np.ndarray) -> np.ndarray:
    R = np.ascontiguousarray(R, dtype=np.float64).reshape(9)
    r = np.zeros(3)
    lib().ref_rodrigues_inv(_p(R, _f64p), _p(r, _f64p))
    return r


def project_points(P3, rvec, tvec, K, dist):
    P3 = np.ascontiguousarray(P3, dtype=np.float64)
    rvec = np.ascontiguousarray(rvec, dtype=np.float64).reshape(3)
    tvec = np.ascontiguousarray(tvec, dtype=np.float64).reshape(3)
    K = np.ascontiguousarray(K, dtype=np.float64)
    dist = np.ascontiguousarray(np.resize(np.asarray(dist, np.float64), 5))
    uv = np.zeros((len(P3), 2))
    lib().ref_project_points(_p(P3, _f64p), len(P3), _p(rvec, _f64p), _p(tvec, _f64p), _p(K, _f64p),
                             _p(dist, _f64p), _p(uv, _f64p))
    return uv


def frame_pose(prevL, prevR, curL, K, dist, baseline, nfeatures=500):
    """One stereo_slam.py ORB-branch iteration (:232-303).  Returns a dict with every
    intermediate (for parity tests) and the 4x4 relative transform (or None)."""
    kp0, d0 = orb_detect_compute(prevL, nfeatures)
    kp1, d1 = orb_detect_compute(curL, nfeatures)
    m = bf_match(d0, d1) if len(d0) and len(d1) else np.zeros((0, 3), np.int32)
    mk0 = kp0[:, :2].astype(np.float32)[m[:, 0]]
    mk1 = kp1[:, :2].astype(np.float32)[m[:, 1]]
    disp16 = sgbm(prevL, prevR)
    disp = disparity_map(disp16)
    P3, p2, valid = backproject(disp, mk0, mk1, K, baseline)
    out = dict(kp0=kp0, d0=d0, kp1=kp1, d1=d1, matches=m, disp16=disp16, P3=P3, p2=p2, T=None)
    if len(P3) >= 6:
        ok, rv, tv, inl, ni, bg = solve_pnp_ransac(P3, p2, K, dist)
        out.update(ok=ok, rvec=rv, tvec=tv, inliers=inl)
        T = np.eye(4)
        T[:3, :3] = rodrigues(rv)
        T[:3, 3] = tv
        out["T"] = T
    return out
