"""cv2-shaped faces of libfvo (face 1) and a SuperGlue-`Matching`-shaped
callable (face 2), so the reference's lines run unchanged on the MI355X path.

Face 1 mirrors the OpenCV calls of ros_ws/src/stereo_slam.py:
    orb = ORB_create()                                          (:84)
    bf = BFMatcher(NORM_HAMMING, crossCheck=True)               (:85)
    kps, desc = orb.detectAndCompute(img, None)                 (:232-233, :240-241)
    matches = bf.match(desc0, desc1)                            (:234, :242)
    StereoSGBM_create(...).compute(L, R)                        (:108-117)
    ok, rvec, tvec, inliers = solvePnPRansac(P, p, K, dist, ...)  (:294-295)
    R, _ = Rodrigues(rvec)                                      (:298)
and of ros_ws/src/mono_slam.py:
    E, mask = findEssentialMat(m0, m1, focal=, pp=, method=RANSAC, prob=0.999, threshold=1.0)  (:111)
    _, R, t, _ = recoverPose(E, m0, m1, focal=, pp=)            (:112)
Face 2 mirrors `feature_matcher({'image0': t0, 'image1': t1})` (:81, :210-229) with
ORB + BF-cross-check underneath; matching_scores0 = 1 - distance/256.

Inputs may be NumPy arrays (host) or torch tensors (host or device); outputs follow
OpenCV's types (tuples of KeyPoint, lists of DMatch, NumPy arrays).  Every computation runs
in libfvo on the GPU; there is no CPU fallback (a missing GPU or library raises).
Unsupported parameter values raise NotImplementedError instead of silently differing."""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

NORM_HAMMING = 6
ORB_HARRIS_SCORE = 0
STEREO_SGBM_MODE_SGBM = 0
STEREO_SGBM_MODE_HH = 1
STEREO_SGBM_MODE_SGBM_3WAY = 2
SOLVEPNP_ITERATIVE = 0
RANSAC = 8


class error(RuntimeError):
    """Raised where OpenCV raises cv2.error."""


class KeyPoint:
    __slots__ = ("pt", "size", "angle", "response", "octave", "class_id")

    def __init__(self, x=0.0, y=0.0, size=0.0, angle=-1.0, response=0.0, octave=0, class_id=-1):
        self.pt = (float(x), float(y))
        self.size, self.angle, self.response = float(size), float(angle), float(response)
        self.octave, self.class_id = int(octave), int(class_id)

    def __repr__(self):
        return f"KeyPoint(pt={self.pt}, size={self.size}, angle={self.angle:.3f}, octave={self.octave})"


class DMatch:
    __slots__ = ("queryIdx", "trainIdx", "imgIdx", "distance")

    def __init__(self, queryIdx=-1, trainIdx=-1, imgIdx=0, distance=float("inf")):
        self.queryIdx, self.trainIdx, self.imgIdx, self.distance = int(queryIdx), int(trainIdx), imgIdx, float(distance)

    def __repr__(self):
        return f"DMatch({self.queryIdx}->{self.trainIdx}, d={self.distance:g})"


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("forest_slam_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
    return torch.device("cuda", torch.cuda.current_device())


def _u8_image(img, name="image") -> torch.Tensor:
    t = img if isinstance(img, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(img))
    if t.dtype != torch.uint8:
        raise error(f"{name}: expected an 8-bit single-channel image, got {t.dtype}")
    if t.dim() != 2:
        raise error(f"{name}: expected a single-channel (H, W) image, got shape {tuple(t.shape)}")
    return t.to(_device()).contiguous()


class _CtxCache:
    """Contexts are created once per (size, params) and reused (no allocation per call)."""

    def __init__(self):
        self._ctx = {}

    def get(self, key, factory):
        c = self._ctx.get(key)
        if c is None:
            c = self._ctx[key] = factory()
        return c


# --------------------------------------------------------------------------- ORB
class ORB:
    """cv2.ORB (detector + rBRIEF extractor); only the reference's configuration family
    is implemented: firstLevel 0, WTA_K 2, HARRIS_SCORE, patchSize 31."""

    def __init__(self, nfeatures=500, scaleFactor=1.2, nlevels=8, edgeThreshold=31, firstLevel=0, WTA_K=2,
                 scoreType=ORB_HARRIS_SCORE, patchSize=31, fastThreshold=20):
        if firstLevel != 0 or WTA_K != 2 or scoreType != ORB_HARRIS_SCORE or patchSize != 31:
            raise NotImplementedError("ORB: only firstLevel=0, WTA_K=2, HARRIS_SCORE, patchSize=31 are implemented")
        self.params = dict(nfeatures=int(nfeatures), scale_factor=float(scaleFactor), nlevels=int(nlevels),
                           edge_threshold=int(edgeThreshold), fast_threshold=int(fastThreshold))
        self._cache = _CtxCache()

    def _context(self, W, H):
        key = (W, H)
        return self._cache.get(key, lambda: _lib.Context(W, H, max_batch=1, stages=_lib.STAGE_ORB, **self.params))

    def detectAndComputeDevice(self, img):
        """Device-side variant: (kp f32[N,8] records, desc u8[N,32]) as torch tensors."""
        t = _u8_image(img)
        H, W = t.shape
        ctx = self._context(W, H)
        kp, desc, cnt = ctx.orb(t)
        n = int(cnt[0].item())
        if n < 0:
            raise error(f"ORB: keypoint capacity {ctx.kp_cap} exceeded (needs {-n})")
        return kp[0, :n], desc[0, :n]

    def detectAndCompute(self, image, mask=None, descriptors=None, useProvidedKeypoints=False):
        if mask is not None or useProvidedKeypoints:
            raise NotImplementedError("ORB.detectAndCompute: mask / provided keypoints are not implemented")
        kp, desc = self.detectAndComputeDevice(image)
        rec = kp.cpu().numpy()
        kps = tuple(KeyPoint(r[0], r[1], r[2], r[3], r[4], int(r[5]), int(r[6])) for r in rec)
        d = desc.cpu().numpy()
        return kps, (d if len(kps) else None)

    def detect(self, image, mask=None):
        return self.detectAndCompute(image, mask)[0]

    def getMaxFeatures(self):
        return self.params["nfeatures"]


def ORB_create(nfeatures=500, scaleFactor=1.2, nlevels=8, edgeThreshold=31, firstLevel=0, WTA_K=2,
               scoreType=ORB_HARRIS_SCORE, patchSize=31, fastThreshold=20):
    return ORB(nfeatures, scaleFactor, nlevels, edgeThreshold, firstLevel, WTA_K, scoreType, patchSize, fastThreshold)


# --------------------------------------------------------------------------- BFMatcher
def _desc_tensor(d, name):
    if d is None:
        raise error(f"BFMatcher.match: {name} descriptors are empty (None)")
    t = d if isinstance(d, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(d))
    if t.dtype != torch.uint8 or t.dim() != 2 or (t.shape[0] > 0 and t.shape[1] != 32):
        raise error(f"BFMatcher.match: {name} must be uint8 [N, 32] (ORB descriptors), got {tuple(t.shape)} {t.dtype}")
    return t


class BFMatcher:
    """cv2.BFMatcher(NORM_HAMMING, crossCheck=True): mutual nearest neighbours by Hamming
    distance, first index on ties, DMatch list in ascending queryIdx."""

    def __init__(self, normType=NORM_HAMMING, crossCheck=False):
        if normType != NORM_HAMMING or not crossCheck:
            raise NotImplementedError("BFMatcher: only NORM_HAMMING with crossCheck=True is implemented")
        self._ctx = None

    def _context(self, n):
        cap = max(1024, -(-n // 1024) * 1024)
        if self._ctx is None or self._ctx.kp_cap < n:
            self._ctx = _lib.Context(64, 64, max_batch=1, stages=_lib.STAGE_BF, kp_capacity=cap)
        return self._ctx

    def matchDevice(self, d0: torch.Tensor, d1: torch.Tensor):
        """Device-side variant: int32 [M,3] rows (queryIdx, trainIdx, distance)."""
        dev = _device()
        n0, n1 = d0.shape[0], d1.shape[0]
        if n0 == 0 or n1 == 0:
            return torch.empty((0, 3), dtype=torch.int32, device=dev)
        ctx = self._context(max(n0, n1))
        cap = ctx.kp_cap
        q = torch.zeros((1, cap, 32), dtype=torch.uint8, device=dev)
        t = torch.zeros((1, cap, 32), dtype=torch.uint8, device=dev)
        q[0, :n0] = d0.to(dev)
        t[0, :n1] = d1.to(dev)
        nq = torch.tensor([n0], dtype=torch.int32, device=dev)
        nt = torch.tensor([n1], dtype=torch.int32, device=dev)
        m, nm = ctx.bf_match(q, nq, t, nt)
        return m[0, :int(nm[0].item())]

    def match(self, queryDescriptors, trainDescriptors, mask=None):
        if mask is not None:
            raise NotImplementedError("BFMatcher.match: mask is not implemented")
        m = self.matchDevice(_desc_tensor(queryDescriptors, "query"), _desc_tensor(trainDescriptors, "train"))
        return [DMatch(r[0], r[1], 0, float(r[2])) for r in m.cpu().numpy()]


def BFMatcher_create(normType=NORM_HAMMING, crossCheck=False):
    return BFMatcher(normType, crossCheck)


# --------------------------------------------------------------------------- StereoSGBM
class StereoSGBM:
    """cv2.StereoSGBM in MODE_SGBM_3WAY (the reference's mode).  compute() returns int16
    disparity x16 with (minDisparity-1)*16 for invalid pixels, after OpenCV's 3x3 median."""

    def __init__(self, minDisparity=0, numDisparities=16, blockSize=3, P1=0, P2=0, disp12MaxDiff=0, preFilterCap=0,
                 uniquenessRatio=0, speckleWindowSize=0, speckleRange=0, mode=STEREO_SGBM_MODE_SGBM):
        if mode != STEREO_SGBM_MODE_SGBM_3WAY:
            raise NotImplementedError("StereoSGBM: only mode=STEREO_SGBM_MODE_SGBM_3WAY is implemented")
        if blockSize != 7 or numDisparities not in (64, 96, 128) or uniquenessRatio != 0 or speckleWindowSize != 0:
            raise NotImplementedError("StereoSGBM: implemented for blockSize=7, numDisparities in {64, 96, 128}, "
                                      "uniquenessRatio=0, speckleWindowSize=0")
        self.params = dict(min_disparity=int(minDisparity), num_disparities=int(numDisparities),
                           block_size=int(blockSize), P1=int(P1), P2=int(P2), disp12_max_diff=int(disp12MaxDiff),
                           pre_filter_cap=int(preFilterCap), uniqueness_ratio=int(uniquenessRatio))
        self._cache = _CtxCache()

    def computeDevice(self, left, right) -> torch.Tensor:
        L, R = _u8_image(left, "left"), _u8_image(right, "right")
        if L.shape != R.shape:
            raise error("StereoSGBM.compute: left and right images differ in size")
        H, W = L.shape
        ctx = self._cache.get((W, H), lambda: _lib.Context(W, H, max_batch=1, stages=_lib.STAGE_SGBM,
                                                           **self.params))
        return ctx.sgbm(L, R)[0]

    def compute(self, left, right, disparity=None):
        return self.computeDevice(left, right).cpu().numpy()


# --------------------------------------------------------------------------- motion blur
def blur_centers(height, width, blur_percentage=10, rng=None):
    """The pixels apply_random_motion_blur blurs around (stereo_slam.py:161-165):
    random.sample(range(H*W), int(H*W*(blur_percentage/100.0))).  The reference draws from
    Python's unseeded global `random`; pass a seeded `random.Random` for reproducible runs
    (rng=None uses the global module state, as the reference does)."""
    import random
    n = int((height * width) * (blur_percentage / 100.0))
    return np.asarray((rng or random).sample(range(height * width), n), dtype=np.int32)


_blur_cache = _CtxCache()


def apply_random_motion_blur(image, blur_percentage=10, kernel_size=15, angle=0, rng=None, centers=None):
    """stereo_slam.py:157-178 on the GPU (fvo_motion_blur): blur the whole image with the
    k-tap motion kernel (apply_motion_blur, :142-154) and keep it inside the union of the
    squares around the sampled pixels.  `centers` overrides the sampling (flat indices)."""
    if angle != 0:
        raise NotImplementedError("apply_random_motion_blur: only angle=0 (the reference's value) is implemented")
    img = _u8_image(image)
    H, W = img.shape
    if centers is None:
        centers = blur_centers(H, W, blur_percentage, rng)
    c = torch.from_numpy(np.ascontiguousarray(centers, dtype=np.int32)).to(img.device)[None]
    n = torch.tensor([c.shape[1]], dtype=torch.int32, device=img.device)
    ctx = _blur_cache.get((W, H), lambda: _lib.Context(W, H, max_batch=1, stages=_lib.STAGE_BF,
                                                                   kp_capacity=64))
    out, _ = ctx.motion_blur(img, kernel_size, c if c.shape[1] else None, n, angle=float(angle))
    return out[0].cpu().numpy()


def StereoSGBM_create(minDisparity=0, numDisparities=16, blockSize=3, P1=0, P2=0, disp12MaxDiff=0, preFilterCap=0,
                      uniquenessRatio=0, speckleWindowSize=0, speckleRange=0, mode=STEREO_SGBM_MODE_SGBM):
    return StereoSGBM(minDisparity, numDisparities, blockSize, P1, P2, disp12MaxDiff, preFilterCap, uniquenessRatio,
                      speckleWindowSize, speckleRange, mode)


# --------------------------------------------------------------------------- solvePnPRansac
_pnp_cache = _CtxCache()


def solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs, rvec=None, tvec=None,
                   useExtrinsicGuess=False, iterationsCount=100, reprojectionError=8.0, confidence=0.99,
                   inliers=None, flags=SOLVEPNP_ITERATIVE):
    """cv2.solvePnPRansac(flags=SOLVEPNP_ITERATIVE) -> (retval, rvec (3,1), tvec (3,1), inliers (k,1) | None).
    Object points are taken as float32 (OpenCV converts them so).  Sets of fewer than 6
    points return (False, zeros, zeros, None): the reference never calls with fewer
    (stereo_slam.py:292), and the kernel applies that guard."""
    if useExtrinsicGuess or flags != SOLVEPNP_ITERATIVE:
        raise NotImplementedError("solvePnPRansac: only SOLVEPNP_ITERATIVE without extrinsic guess is implemented")
    P = np.ascontiguousarray(np.asarray(objectPoints, dtype=np.float32).reshape(-1, 3))
    p = np.ascontiguousarray(np.asarray(imagePoints, dtype=np.float32).reshape(-1, 2))
    if P.shape[0] != p.shape[0]:
        raise error("solvePnPRansac: object and image point counts differ")
    K = np.asarray(cameraMatrix, dtype=np.float64).reshape(3, 3)
    dist = np.zeros(5) if distCoeffs is None else np.asarray(distCoeffs, dtype=np.float64).reshape(-1)
    if dist.size > 5 and np.any(dist[5:] != 0):
        raise NotImplementedError("solvePnPRansac: only (k1, k2, p1, p2[, k3]) distortion is implemented")
    n = P.shape[0]
    dev = _device()
    cap = max(1024, -(-n // 1024) * 1024)
    ctx = _pnp_cache.get(cap, lambda: _lib.Context(64, 64, max_batch=1, stages=_lib.STAGE_POSE, kp_capacity=cap))
    P3 = torch.zeros((1, cap, 3), dtype=torch.float32, device=dev)
    p2 = torch.zeros((1, cap, 2), dtype=torch.float32, device=dev)
    P3[0, :n] = torch.from_numpy(P).to(dev)
    p2[0, :n] = torch.from_numpy(p).to(dev)
    cnt = torch.tensor([n], dtype=torch.int32, device=dev)
    rv, tv, T, st, inl = ctx.pnp_ransac(P3, p2, cnt, K, dist[:5], reproj=float(reprojectionError),
                                        confidence=float(confidence), iterations=int(iterationsCount))
    rv, tv = rv[0].cpu().numpy().reshape(3, 1), tv[0].cpu().numpy().reshape(3, 1)
    if int(st[0].item()) != 1:
        return False, np.zeros((3, 1)), np.zeros((3, 1)), None
    idx = np.nonzero(inl[0, :n].cpu().numpy())[0].astype(np.int32).reshape(-1, 1)
    return True, rv, tv, idx



_mono_cache = _CtxCache()


def _mono_ctx(n):
    cap = max(1024, -(-n // 1024) * 1024)
    return cap, _mono_cache.get(cap, lambda: _lib.Context(64, 64, max_batch=1, stages=_lib.STAGE_MONO,
                                                          kp_capacity=cap))


def _pinhole(cameraMatrix, focal, pp, name):
    if cameraMatrix is not None:
        K = np.asarray(cameraMatrix, dtype=np.float64).reshape(3, 3)
        if K[0, 0] != K[1, 1]:
            raise NotImplementedError(f"{name}: only fx == fy camera matrices are implemented")
        return float(K[0, 0]), (float(K[0, 2]), float(K[1, 2]))
    return float(focal), (float(pp[0]), float(pp[1]))


def _point_pairs(points1, points2, name):
    p0 = np.ascontiguousarray(np.asarray(points1, dtype=np.float32).reshape(-1, 2))
    p1 = np.ascontiguousarray(np.asarray(points2, dtype=np.float32).reshape(-1, 2))
    if p0.shape[0] != p1.shape[0]:
        raise error(f"{name}: point counts differ")
    n = p0.shape[0]
    cap, ctx = _mono_ctx(n)
    dev = _device()
    P0 = torch.zeros((1, cap, 2), dtype=torch.float32, device=dev)
    P1 = torch.zeros((1, cap, 2), dtype=torch.float32, device=dev)
    P0[0, :n] = torch.from_numpy(p0).to(dev)
    P1[0, :n] = torch.from_numpy(p1).to(dev)
    return n, ctx, P0, P1, torch.tensor([n], dtype=torch.int32, device=dev)


def findEssentialMat(points1, points2, cameraMatrix=None, method=RANSAC, prob=0.999, threshold=1.0, maxIters=1000,
                     mask=None, focal=1.0, pp=(0.0, 0.0)):
    """cv2.findEssentialMat(points1, points2, focal=, pp=, method=RANSAC, prob=, threshold=)
    (mono_slam.py:111) -> (E (3,3) f64, mask (n,1) u8), or (None, None) when RANSAC finds no
    model / fewer than 5 points are given."""
    if method != RANSAC:
        raise NotImplementedError("findEssentialMat: only method=RANSAC is implemented")
    f, c = _pinhole(cameraMatrix, focal, pp, "findEssentialMat")
    n, ctx, P0, P1, cnt = _point_pairs(points1, points2, "findEssentialMat")
    if maxIters > 1000:
        raise NotImplementedError("findEssentialMat: maxIters > 1000")
    E, m, st = ctx.find_essential(P0, P1, cnt, f, c, prob=float(prob), threshold=float(threshold),
                                  max_iters=int(maxIters))
    st = int(st[0].item())
    if st == -2:
        raise NotImplementedError("findEssentialMat: 5 points with several solutions (stacked E)")
    if st != 1:
        return None, None
    return E[0].cpu().numpy(), m[0, :n].cpu().numpy().reshape(-1, 1)


def recoverPose(E, points1, points2, cameraMatrix=None, R=None, t=None, focal=1.0, pp=(0.0, 0.0), mask=None):
    """cv2.recoverPose(E, points1, points2, focal=, pp=) (mono_slam.py:112) ->
    (n_good, R (3,3), t (3,1), mask); distanceThresh 50 as in that OpenCV overload."""
    if mask is not None:
        raise NotImplementedError("recoverPose: an input mask is not implemented (the reference passes none)")
    E = np.asarray(E, dtype=np.float64)
    if E.shape != (3, 3):
        raise error("recoverPose: E must be 3x3")
    f, c = _pinhole(cameraMatrix, focal, pp, "recoverPose")
    n, ctx, P0, P1, cnt = _point_pairs(points1, points2, "recoverPose")
    Et = torch.from_numpy(np.ascontiguousarray(E)).to(P0.device)[None]
    Rm, tv, T, g = ctx.recover_pose(Et, P0, P1, cnt, f, c)
    return int(g[0].item()), Rm[0].cpu().numpy(), tv[0].cpu().numpy().reshape(3, 1), None

def Rodrigues(src):
    """cv2.Rodrigues for a rotation vector (3,1)/(1,3)/(3,) -> (R 3x3, jacobian 3x9), or a
    rotation matrix -> (rvec 3x1, None: that jacobian is not implemented).  Host arithmetic on 3x3 values, as the
    reference does it on the host (stereo_slam.py:298)."""
    a = np.asarray(src, dtype=np.float64)
    if a.size == 3:
        return _rodrigues_vec(a.reshape(3))
    if a.shape == (3, 3):
        return _rodrigues_mat(a)
    raise error("Rodrigues: input must be a 3-vector or a 3x3 matrix")


def _rodrigues_vec(r):
    th = float(np.sqrt(r @ r))
    J = np.zeros((3, 9))
    if th < np.finfo(np.float64).eps:
        # OpenCV's constant for theta = 0 (sign convention kept as OpenCV has it)
        J[0, 5] = J[1, 6] = J[2, 1] = 1
        J[0, 7] = J[1, 2] = J[2, 3] = -1
        return np.eye(3), J
    c, s = np.cos(th), np.sin(th)
    c1 = 1.0 - c
    itheta = 1.0 / th
    k = r * itheta
    rrt = np.outer(k, k)
    rx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    R = c * np.eye(3) + c1 * rrt + s * rx
    # d(R)/d(r), OpenCV's closed form (row-major R, 3 x 9)
    I = np.eye(3).reshape(-1)
    drrt = np.array([[k[0] + k[0], k[1], k[2], k[1], 0, 0, k[2], 0, 0],
                     [0, k[0], 0, k[0], k[1] + k[1], k[2], 0, k[2], 0],
                     [0, 0, k[0], 0, 0, k[1], k[0], k[1], k[2] + k[2]]])
    d_r_x_ = np.array([[0, 0, 0, 0, 0, -1, 0, 1, 0], [0, 0, 1, 0, 0, 0, -1, 0, 0], [0, -1, 0, 1, 0, 0, 0, 0, 0]])
    rrt_f, rx_f = rrt.reshape(-1), rx.reshape(-1)
    for i in range(3):
        ri = k[i]
        a0, a1, a3 = -s * ri, (s - 2 * c1 * itheta) * ri, c1 * itheta
        a2, a4 = (c - s * itheta) * ri, s * itheta
        J[i] = a0 * I + a1 * rrt_f + a2 * rx_f + a3 * drrt[i] + a4 * d_r_x_[i]
    return R, J


def _rodrigues_mat(R):
    U, _, Vt = np.linalg.svd(R)
    R = U @ Vt
    r = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    s = np.sqrt((r @ r) * 0.25)
    c = np.clip((np.trace(R) - 1) * 0.5, -1.0, 1.0)
    th = np.arccos(c)
    if s < 1e-5:
        if c > 0:
            return np.zeros((3, 1)), None
        t = (np.diag(R) + 1) * 0.5
        r = np.sqrt(np.maximum(t, 0))
        if R[0, 1] < 0:
            r[1] = -r[1]
        if R[0, 2] < 0:
            r[2] = -r[2]
        if abs(r[0]) < abs(r[1]) and abs(r[0]) < abs(r[2]) and (R[1, 2] > 0) != (r[1] * r[2] > 0):
            r[2] = -r[2]
        r = r * (th / np.sqrt(r @ r))
        return r.reshape(3, 1), None
    r = r * ((1.0 / (2 * s)) * th)
    return r.reshape(3, 1), None


# --------------------------------------------------------------------------- Matching face
class ORBMatching(torch.nn.Module):
    """Drop-in for SuperGlue's `Matching` as called at stereo_slam.py:81/:210: takes
    {'image0': f32[B,1,H,W] in [0,1], 'image1': ...} and returns per-image lists of
    keypoints0/1 [N,2], scores0/1 [N], descriptors0/1 [32,N] (u8), matches0/1 [N] (int64,
    -1 unmatched) and matching_scores0/1 [N] (1 - distance/256), so `v[0]` picks image 0
    of the batch exactly as the reference does.  ORB + BF-cross-check underneath, one
    batched launch per stage."""

    def __init__(self, config=None, nfeatures=500, **orb_params):
        super().__init__()
        cfg = dict(config or {})
        self.nfeatures = int(cfg.get("nfeatures", nfeatures))
        self.orb_params = orb_params
        self._cache = _CtxCache()

    @staticmethod
    def _to_u8(t: torch.Tensor) -> torch.Tensor:
        # the reference builds the tensors as float32(frame / 255.); this inverts that exactly
        return (t.to(torch.float32) * 255.0).round().clamp_(0, 255).to(torch.uint8)

    def forward(self, data: dict) -> dict:
        i0, i1 = data["image0"], data["image1"]
        if i0.dim() != 4 or i0.shape[1] != 1 or i0.shape != i1.shape:
            raise error("ORBMatching: image0/image1 must both be [B,1,H,W]")
        B, _, H, W = i0.shape
        dev = _device()
        imgs = torch.cat([self._to_u8(i0[:, 0]), self._to_u8(i1[:, 0])]).to(dev).contiguous()
        ctx = self._cache.get((W, H, B), lambda: _lib.Context(W, H, max_batch=2 * B, nfeatures=self.nfeatures,
                                                              stages=_lib.STAGE_ORB | _lib.STAGE_BF,
                                                              **self.orb_params))
        kp, desc, cnt = ctx.orb(imgs)
        m, nm = ctx.bf_match(desc[:B], cnt[:B], desc[B:], cnt[B:])
        cnt_h, nm_h, m_h = cnt.cpu(), nm.cpu(), m.cpu()
        out = {k: [] for k in ("keypoints0", "keypoints1", "scores0", "scores1", "descriptors0", "descriptors1",
                               "matches0", "matches1", "matching_scores0", "matching_scores1")}
        for b in range(B):
            n0, n1 = int(cnt_h[b]), int(cnt_h[B + b])
            if n0 < 0 or n1 < 0:
                raise error(f"ORBMatching: keypoint capacity {ctx.kp_cap} exceeded")
            rows = m_h[b, :int(nm_h[b])].long()
            m0 = torch.full((n0,), -1, dtype=torch.int64)
            m1 = torch.full((n1,), -1, dtype=torch.int64)
            s0 = torch.zeros(n0)
            s1 = torch.zeros(n1)
            if rows.numel():
                m0[rows[:, 0]] = rows[:, 1]
                m1[rows[:, 1]] = rows[:, 0]
                sc = 1.0 - rows[:, 2].float() / 256.0
                s0[rows[:, 0]] = sc
                s1[rows[:, 1]] = sc
            out["keypoints0"].append(kp[b, :n0, :2])
            out["keypoints1"].append(kp[B + b, :n1, :2])
            out["scores0"].append(kp[b, :n0, 4])
            out["scores1"].append(kp[B + b, :n1, 4])
            out["descriptors0"].append(desc[b, :n0].t())
            out["descriptors1"].append(desc[B + b, :n1].t())
            out["matches0"].append(m0.to(dev))
            out["matches1"].append(m1.to(dev))
            out["matching_scores0"].append(s0.to(dev))
            out["matching_scores1"].append(s1.to(dev))
        return out
