"""ctypes binding of libfvo.so (include/fvo.h) with torch tensors as the buffer type.

The product path: every call lands in a hand-written HIP kernel.  There is no CPU
fallback — if the library or the GPU is missing, construction raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# FVO_LIB: an alternative build of the same library (launch-shape experiments, tools/
# build_variant.py); the product path is the in-tree libfvo.so
LIB_PATH = os.environ.get("FVO_LIB") or os.path.join(_HERE, "libfvo.so")

KP_STRIDE = 8
DESC_BYTES = 32

_lib = None


class FvoConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("width", "height", "max_batch", "nfeatures")] + [
        ("scale_factor", ctypes.c_float)] + [(n, ctypes.c_int32) for n in (
            "nlevels", "edge_threshold", "first_level", "wta_k", "score_type", "patch_size", "fast_threshold",
            "min_disparity", "num_disparities", "block_size", "P1", "P2", "disp12_max_diff", "pre_filter_cap",
            "uniqueness_ratio", "sgbm_stripes", "kp_capacity", "stages", "ba_window", "ba_max_landmarks",
            "ba_max_obs", "sgbm_max_batch", "sgbm_mode", "sgbm_lanes", "sgbm_cols", "sgbm_handoff_us")]


class FvoRegion(ctypes.Structure):
    """fvo_region of include/fvo.h."""
    _fields_ = [("dst", ctypes.c_void_p), ("src", ctypes.c_void_p), ("bytes", ctypes.c_int64)]


FVO_MAX_REGIONS = 32
ABI_VERSION = 7  # FVO_ABI_VERSION of include/fvo.h
STAGE_ORB, STAGE_BF, STAGE_SGBM, STAGE_POSE, STAGE_BA, STAGE_MONO = 1, 2, 4, 8, 16, 32
SGBM_CLASSIC, SGBM_LPATH = 0, 1  # fvo_config.sgbm_mode
SGBM_OK, SGBM_HANDOFF_TIMEOUT = 0, -1  # fvo_sgbm status values

# name -> (restype, argtypes); mirrors include/fvo.h
_P = ctypes.c_void_p
_I = ctypes.c_int32
_L = ctypes.c_int64
SIGNATURES = {
    "fvo_abi_version": (ctypes.c_int, []),
    "fvo_config_default": (None, [ctypes.POINTER(FvoConfig), _I, _I]),
    "fvo_config_size": (ctypes.c_int32, []),
    "fvo_config_offset": (ctypes.c_int32, [ctypes.c_char_p]),
    "fvo_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(FvoConfig), ctypes.POINTER(_P)]),
    "fvo_destroy": (None, [_P]),
    "fvo_last_error": (ctypes.c_char_p, [_P]),
    "fvo_kp_capacity": (ctypes.c_int, [_P]),
    "fvo_workspace_bytes": (ctypes.c_int64, [_P]),
    "fvo_orb_detect_compute": (ctypes.c_int, [_P, _P, _I, _L, _I, _P, _P, _P, _I, _P]),
    "fvo_bf_match": (ctypes.c_int, [_P, _P, _P, _P, _P, _I, _I, _P, _P, _P]),
    "fvo_sgbm": (ctypes.c_int, [_P, _P, _P, _I, _L, _I, _P, _P, _P]),
    "fvo_backproject": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I, _I, _P, ctypes.c_double, _P, _P, _P, _P]),
    "fvo_pnp_ransac": (ctypes.c_int, [_P, _P, _P, _P, _I, _I, _P, _P, ctypes.c_float, ctypes.c_double, _I, _P, _P,
                                      _P, _P, _P, _P]),
    "fvo_keypoint_stereo": (ctypes.c_int, [_P, _P, _P, _P, _I, _I, _P, ctypes.c_double, _P, _P]),
    "fvo_ba_windows": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, ctypes.c_double, _P, _I, _I,
                                      _P, _P, _P]),
    "fvo_ba_landmarks": (ctypes.c_int, [_P, _I, _P, _P, _P]),
    "fvo_ba_count_births": (ctypes.c_int, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "fvo_gather_matches": (ctypes.c_int, [_P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P]),
    "fvo_find_essential": (ctypes.c_int, [_P, _P, _P, _P, _I, _I, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                          ctypes.c_double, ctypes.c_double, _I, _P, _P, _P, _P]),
    "fvo_recover_pose": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I, _I, ctypes.c_double, ctypes.c_double,
                                        ctypes.c_double, ctypes.c_double, _P, _P, _P, _P, _P]),
    "fvo_undistort_gray": (ctypes.c_int, [_P, _P, _I, _L, _I, _P, _P, _P, _L, _I, _P]),
    "fvo_map_transform": (ctypes.c_int, [_P, _P, _I, _P, _I, _L, _P, _P, _L, _P, _P, _P]),
    "fvo_chain_poses": (ctypes.c_int, [_P, _P, _P, _P, _I, _I, _P, _P, _P, _P]),
    "fvo_copy_regions": (ctypes.c_int, [_P, _I, _P, _P]),
    "fvo_count_guard": (ctypes.c_int, [_P, _P, _P, _I, _I, _P, _I, _P, _P]),
    "fvo_voxel_workspace_bytes": (ctypes.c_int64, [_L]),
    "fvo_voxel_down_sample": (ctypes.c_int, [_P, _P, _L, ctypes.c_double, _P, _L, _P, _P, _P, _P]),
    "fvo_motion_blur": (ctypes.c_int, [_P, _P, _I, _L, _I, _I, ctypes.c_double, _P, _P, _I, _P, _P, _L, _I, _P]),
    "fvo_test_retain_best": (ctypes.c_int, [_P, _P, _I, _I, _P, _P, _P]),
    "fvo_debug_buffer": (ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_int64)]),
    "fvo_kernel_count": (ctypes.c_int, []),
    "fvo_kernel_name": (ctypes.c_char_p, [ctypes.c_int]),
    "fvo_timing_enable": (ctypes.c_int, [_P, ctypes.c_uint64]),
    "fvo_timing_read": (ctypes.c_int, [_P, _P, _P]),
}


def check_config_layout(L) -> None:
    """Refuse a library whose fvo_config layout differs from FvoConfig (size and every
    field offset), so fvo_config_default can never write past the ctypes struct."""
    if L.fvo_config_size() != ctypes.sizeof(FvoConfig):
        raise RuntimeError(f"fvo_config is {L.fvo_config_size()} B in libfvo.so, {ctypes.sizeof(FvoConfig)} B here")
    for name, _ in FvoConfig._fields_:
        if L.fvo_config_offset(name.encode()) != getattr(FvoConfig, name).offset:
            raise RuntimeError(f"fvo_config.{name} offset differs between libfvo.so and the binding")


def kernel_names() -> list[str]:
    L = load()
    return [L.fvo_kernel_name(i).decode() for i in range(L.fvo_kernel_count())]


def load(path: str = LIB_PATH):
    """Load libfvo.so (raises if it is missing: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(path):
            raise RuntimeError(f"libfvo.so not found at {path}: run __graft_entry__.build() "
                               "(python -m forest_slam_amd.build); the HIP path has no CPU fallback")
        L = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.fvo_abi_version() != ABI_VERSION:
            raise RuntimeError("libfvo.so ABI version mismatch")
        check_config_layout(L)
        _lib = L
    return _lib


def _ptr(t: torch.Tensor | None):
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("libfvo takes device tensors")
    return ctypes.c_void_p(t.data_ptr())


def _stream(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _i32(x, dev):
    return torch.as_tensor(x, dtype=torch.int32, device=dev)


class Context:
    """One fvo context (device workspace) for a fixed image size and max batch."""

    def __init__(self, width: int, height: int, max_batch: int = 1, device: int | str | torch.device | None = None,
                 **params):
        if not torch.cuda.is_available():
            raise RuntimeError("forest_slam_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.L = load()
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if dev.type != "cuda":
            raise RuntimeError("device must be a cuda (ROCm) device")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        cfg = FvoConfig()
        self.L.fvo_config_default(ctypes.byref(cfg), width, height)
        cfg.max_batch = max_batch
        for k, v in params.items():
            if not hasattr(cfg, k):
                raise TypeError(f"unknown fvo_config field {k}")
            setattr(cfg, k, v)
        self.cfg = cfg
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            rc = self.L.fvo_create(dev.index, ctypes.byref(cfg), ctypes.byref(h))
        if rc != 0 or not h.value:
            raise RuntimeError("fvo_create failed (see stderr)")
        self.h = h
        self.kp_cap = self.L.fvo_kp_capacity(h)
        self.width, self.height, self.max_batch = width, height, max_batch

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.L.fvo_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise RuntimeError("libfvo: " + self.L.fvo_last_error(self.h).decode())

    @property
    def workspace_bytes(self) -> int:
        return int(self.L.fvo_workspace_bytes(self.h))

    def timing_enable(self, names=None):
        """Bracket launches of the named kernels (all if None, none if []) with HIP events."""
        all_names = kernel_names()
        if names is None:
            mask = (1 << len(all_names)) - 1
        else:
            mask = 0
            for n in names:
                mask |= 1 << all_names.index(n)
        self._check(self.L.fvo_timing_enable(self.h, mask))

    def timing_read(self) -> dict:
        """{kernel: (total_ms, launches)} for the launches recorded since the last read."""
        import numpy as np
        nk = self.L.fvo_kernel_count()
        ms = np.zeros(nk, np.float64)
        cnt = np.zeros(nk, np.int32)
        self._check(self.L.fvo_timing_read(self.h, ms.ctypes.data_as(ctypes.c_void_p),
                                           cnt.ctypes.data_as(ctypes.c_void_p)))
        return {n: (float(ms[i]), int(cnt[i])) for i, n in enumerate(kernel_names()) if cnt[i] > 0}

    # ------------------------------------------------------------------ stages
    def orb(self, images: torch.Tensor, out=None):
        """images u8 [B,H,W] (or [H,W]) on device -> (kp f32[B,cap,8], desc u8[B,cap,32], counts i32[B])."""
        if images.dim() == 2:
            images = images[None]
        if images.dtype != torch.uint8:
            raise TypeError("images must be uint8")
        images = images.contiguous()
        B, H, W = images.shape
        if (H, W) != (self.height, self.width):
            raise ValueError(f"context is {self.width}x{self.height}, got {W}x{H}")
        cap = self.kp_cap
        if out is None:
            kp = torch.empty((B, cap, KP_STRIDE), dtype=torch.float32, device=self.device)
            desc = torch.empty((B, cap, DESC_BYTES), dtype=torch.uint8, device=self.device)
            cnt = torch.empty((B,), dtype=torch.int32, device=self.device)
        else:
            kp, desc, cnt = out
        self._check(self.L.fvo_orb_detect_compute(self.h, _ptr(images), B, H * W, W, _ptr(kp), _ptr(desc),
                                                  _ptr(cnt), cap, _stream(self.device)))
        return kp, desc, cnt

    def bf_match(self, d0, n0, d1, n1, out=None):
        """Cross-checked Hamming matching; d* u8 [B,cap,32], n* i32 [B]."""
        B, cap = d0.shape[0], d0.shape[1]
        if out is None:
            m = torch.empty((B, cap, 3), dtype=torch.int32, device=self.device)
            nm = torch.empty((B,), dtype=torch.int32, device=self.device)
        else:
            m, nm = out
        self._check(self.L.fvo_bf_match(self.h, _ptr(d0.contiguous()), _ptr(n0), _ptr(d1.contiguous()), _ptr(n1), B,
                                        cap, _ptr(m), _ptr(nm), _stream(self.device)))
        return m, nm

    def sgbm(self, left, right, out=None, status=None):
        """StereoSGBM 3-way + medianBlur(3) of u8 [B,H,W] pairs -> int16 [B,H,W] disparity*16.
        status: optional int32 [B] device tensor, written SGBM_OK / SGBM_HANDOFF_TIMEOUT."""
        if left.dim() == 2:
            left, right = left[None], right[None]
        left, right = left.contiguous(), right.contiguous()
        B, H, W = left.shape
        if out is None:
            out = torch.empty((B, H, W), dtype=torch.int16, device=self.device)
        if status is not None and (status.dtype != torch.int32 or status.numel() < B or not status.is_contiguous()):
            raise TypeError("status must be a contiguous int32 tensor of >= batch entries")
        self._check(self.L.fvo_sgbm(self.h, _ptr(left), _ptr(right), B, H * W, W, _ptr(out), _ptr(status),
                                    _stream(self.device)))
        return out

    def backproject(self, disp, kp0, kp1, matches, nmatch, K, baseline, out=None):
        B, cap = matches.shape[0], matches.shape[1]
        if out is None:
            P3 = torch.empty((B, cap, 3), dtype=torch.float32, device=self.device)
            p2 = torch.empty((B, cap, 2), dtype=torch.float32, device=self.device)
            n = torch.empty((B,), dtype=torch.int32, device=self.device)
        else:
            P3, p2, n = out
        Kh = (ctypes.c_double * 9)(*[float(v) for v in K.reshape(-1)])
        self._check(self.L.fvo_backproject(self.h, _ptr(disp), _ptr(kp0), _ptr(kp1), _ptr(matches), _ptr(nmatch), B,
                                           cap, Kh, float(baseline), _ptr(P3), _ptr(p2), _ptr(n),
                                           _stream(self.device)))
        return P3, p2, n

    def pnp_ransac(self, P3, p2, n, K, dist, reproj=1.0, confidence=0.99, iterations=1000, out=None):
        B, cap = P3.shape[0], P3.shape[1]
        if out is None:
            rvec = torch.empty((B, 3), dtype=torch.float64, device=self.device)
            tvec = torch.empty((B, 3), dtype=torch.float64, device=self.device)
            T = torch.empty((B, 4, 4), dtype=torch.float64, device=self.device)
            st = torch.empty((B,), dtype=torch.int32, device=self.device)
            inl = torch.empty((B, cap), dtype=torch.uint8, device=self.device)
        else:
            rvec, tvec, T, st, inl = out
        Kh = (ctypes.c_double * 9)(*[float(v) for v in K.reshape(-1)])
        dh = (ctypes.c_double * 5)(*([float(v) for v in list(dist)[:5]] + [0.0] * (5 - min(5, len(dist)))))
        self._check(self.L.fvo_pnp_ransac(self.h, _ptr(P3), _ptr(p2), _ptr(n), B, cap, Kh, dh, float(reproj),
                                          float(confidence), int(iterations), _ptr(rvec), _ptr(tvec), _ptr(T),
                                          _ptr(st), _ptr(inl), _stream(self.device)))
        return rvec, tvec, T, st, inl

    def keypoint_stereo(self, disp, kp, nkp, K, baseline, out=None):
        """Stereo point (X, Y, Z, d) of every keypoint (fvo_keypoint_stereo); Z = 0 invalid."""
        B, cap = kp.shape[0], kp.shape[1]
        if out is None:
            out = torch.empty((B, cap, 4), dtype=torch.float32, device=self.device)
        Kh = (ctypes.c_double * 9)(*[float(v) for v in K.reshape(-1)])
        self._check(self.L.fvo_keypoint_stereo(self.h, _ptr(disp), _ptr(kp), _ptr(nkp), B, cap, Kh, float(baseline),
                                               _ptr(out), _stream(self.device)))
        return out

    def ba_windows(self, kp, nkp, matches, nmatch, stereo, T_rel, first_end, n_windows, first_valid, K, baseline,
                   iterations=10, scale_factor=1.2, out=None):
        """Windowed local BA over frame arrays [F,...] (fvo_ba_windows).  Observation
        weights 1 / scale_factor^(2 octave) (scale_factor as a Python float, the value
        ORB_create() receives).  Returns (T_out f64[n_windows,4,4] refined last-pair
        transforms, stats f64[n_windows,6])."""
        F, cap = kp.shape[0], kp.shape[1]
        if out is None:
            Tout = torch.empty((n_windows, 4, 4), dtype=torch.float64, device=self.device)
            stats = torch.empty((n_windows, 6), dtype=torch.float64, device=self.device)
        else:
            Tout, stats = out
        Kh = (ctypes.c_double * 9)(*[float(v) for v in K.reshape(-1)])
        nl = int(self.cfg.nlevels)
        isig = (ctypes.c_double * nl)(*[1.0 / (float(scale_factor) ** (2 * o)) for o in range(nl)])
        self._check(self.L.fvo_ba_windows(self.h, _ptr(kp), _ptr(nkp), _ptr(matches), _ptr(nmatch), _ptr(stereo),
                                          _ptr(T_rel), F, cap, int(first_end), int(n_windows), int(first_valid), Kh,
                                          float(baseline), isig, nl, int(iterations), _ptr(Tout), _ptr(stats),
                                          _stream(self.device)))
        return Tout, stats

    def ba_count_births(self, matches, nmatch, stereo, first_end, n_windows, first_valid):
        """fvo_ba_count_births: the landmark-birth counting of the next ba_windows call with the
        same frame arrays and window range, issued ahead on the current stream (it needs neither
        T_rel nor the keypoints)."""
        F, cap = matches.shape[0], matches.shape[1]
        self._check(self.L.fvo_ba_count_births(self.h, _ptr(matches), _ptr(nmatch), _ptr(stereo), F, cap,
                                               int(first_end), int(n_windows), int(first_valid),
                                               _stream(self.device)))

    def ba_landmarks(self, window: int, out=None):
        """Refined landmarks of one window of the last ba_windows call (device tensors,
        no host sync): (xyz f64[ba_max_landmarks,3], count i32[1])."""
        if out is None:
            xyz = torch.empty((int(self.cfg.ba_max_landmarks), 3), dtype=torch.float64, device=self.device)
            cnt = torch.empty((1,), dtype=torch.int32, device=self.device)
        else:
            xyz, cnt = out
        self._check(self.L.fvo_ba_landmarks(self.h, int(window), _ptr(xyz), _ptr(cnt), _stream(self.device)))
        return xyz, cnt

    def undistort_gray(self, bgr, K, dist, out=None):
        """cv2.undistort + cvtColor(BGR2GRAY): bgr u8 [B,H,W,3] (or [H,W,3]) -> gray u8 [B,H,W]."""
        if bgr.dim() == 3:
            bgr = bgr[None]
        if bgr.dtype != torch.uint8 or bgr.shape[-1] != 3:
            raise TypeError("bgr must be uint8 [B,H,W,3]")
        bgr = bgr.contiguous()
        B, H, W, _ = bgr.shape
        if (H, W) != (self.height, self.width):
            raise ValueError(f"context is {self.width}x{self.height}, got {W}x{H}")
        if out is None:
            out = torch.empty((B, H, W), dtype=torch.uint8, device=self.device)
        Kh = (ctypes.c_double * 9)(*[float(v) for v in np.asarray(K, np.float64).reshape(-1)])
        d = [float(v) for v in np.asarray(dist, np.float64).reshape(-1)[:5]]
        dh = (ctypes.c_double * 5)(*(d + [0.0] * (5 - len(d))))
        self._check(self.L.fvo_undistort_gray(self.h, _ptr(bgr), B, H * W * 3, W * 3, Kh, dh, _ptr(out), H * W, W,
                                              _stream(self.device)))
        return out

    def motion_blur(self, img, ksize, centers=None, n_centers=None, angle=0.0, out=None, mask=None):
        """apply_random_motion_blur (stereo_slam.py:142-178) on gray u8 [B,H,W] images.
        centers: i32 [B,cap] flat pixel indices on the device (or None: no blurred pixel),
        n_centers: i32 [B] device counts.  Returns (out u8 [B,H,W], mask u8 [B,H,W])."""
        if img.dim() == 2:
            img = img[None]
        if img.dtype != torch.uint8:
            raise TypeError("img must be uint8 [B,H,W]")
        img = img.contiguous()
        B, H, W = img.shape
        if (H, W) != (self.height, self.width):
            raise ValueError(f"context is {self.width}x{self.height}, got {W}x{H}")
        if out is None:
            out = torch.empty_like(img)
        if mask is None:
            mask = torch.empty_like(img)
        if centers is None:
            cptr, nptr, cap = None, None, 0
        else:
            if centers.dtype != torch.int32 or n_centers is None or n_centers.dtype != torch.int32:
                raise TypeError("centers / n_centers must be int32 device tensors")
            centers, n_centers = centers.contiguous(), n_centers.contiguous()
            if centers.dim() != 2 or centers.shape[0] != B or n_centers.numel() != B:
                raise ValueError("centers must be [B, cap] and n_centers [B]")
            cptr, nptr, cap = _ptr(centers), _ptr(n_centers), int(centers.shape[1])
        self._check(self.L.fvo_motion_blur(self.h, _ptr(img), B, H * W, W, int(ksize), float(angle), cptr, nptr, cap,
                                           _ptr(mask), _ptr(out), H * W, W, _stream(self.device)))
        return out, mask

    def map_transform(self, points, n_points, T, map_count, map_xyz64=None, map_xyz32=None):
        """Append T[b] @ [p; 1] of every set b to the map (stereo_slam.py:308-318; fvo_map_transform).
        points f32 [B,cap,>=3], n_points i32 [B], T f64 [B,4,4] (all device); map_count i32 [1]
        (device, advanced by the call); map_xyz64 f64 [M,3] and/or map_xyz32 f32 [M,3]."""
        if points.dtype != torch.float32 or points.dim() != 3 or points.shape[2] < 3:
            raise TypeError("points must be float32 [B, cap, >=3]")
        if map_xyz64 is None and map_xyz32 is None:
            raise ValueError("need map_xyz64 and/or map_xyz32")
        points, T = points.contiguous(), T.to(torch.float64).contiguous()
        B, cap, st = points.shape
        if T.shape != (B, 4, 4) or n_points.dtype != torch.int32 or n_points.numel() != B:
            raise ValueError("T must be [B,4,4] and n_points int32 [B]")
        caps = [m.shape[0] for m in (map_xyz64, map_xyz32) if m is not None]
        self._check(self.L.fvo_map_transform(self.h, _ptr(points), st, _ptr(n_points), B, cap, _ptr(T),
                                             _ptr(map_count), min(caps),
                                             _ptr(map_xyz64) if map_xyz64 is not None else None,
                                             _ptr(map_xyz32) if map_xyz32 is not None else None,
                                             _stream(self.device)))
        return map_count

    def chain_poses(self, T, status, cum_state, n_points=None, out=None):
        """Advance the pose chains of S sequences over one batch of n frames each on the device
        (stereo_slam.py:292-306; fvo_chain_poses).  T f64 [S,n,4,4], status i32 [S,n], n_points
        i32 [S,n] or None, cum_state f64 [S,4,4] (advanced in place).  Returns (cum f64
        [S,n,4,4] = each frame's cumulative pose, n_points_out i32 [S,n] = n_points of the
        posed frames (status >= 0), 0 elsewhere; None without n_points)."""
        if T.dim() != 4 or T.shape[2:] != (4, 4) or T.dtype != torch.float64 or not T.is_contiguous():
            raise TypeError("T must be contiguous float64 [S, n, 4, 4]")
        S, n = T.shape[0], T.shape[1]
        if status.dtype != torch.int32 or status.shape != (S, n) or not status.is_contiguous():
            raise TypeError("status must be contiguous int32 [S, n]")
        if cum_state.dtype != torch.float64 or cum_state.shape != (S, 4, 4) or not cum_state.is_contiguous():
            raise TypeError("cum_state must be contiguous float64 [S, 4, 4]")
        if n_points is not None and (n_points.dtype != torch.int32 or n_points.shape != (S, n)
                                     or not n_points.is_contiguous()):
            raise TypeError("n_points must be contiguous int32 [S, n]")
        if out is None:
            cum = torch.empty_like(T)
            npo = torch.empty_like(n_points) if n_points is not None else None
        else:
            cum, npo = out
        self._check(self.L.fvo_chain_poses(self.h, _ptr(T), _ptr(status), _ptr(n_points), S, n, _ptr(cum_state),
                                           _ptr(cum), _ptr(npo), _stream(self.device)))
        return cum, npo

    def copy_regions(self, pairs):
        """Device-to-device copies ``dst.copy_(src)`` for every (dst, src) in pairs, in list
        order, batched into fvo_copy_regions launches of up to FVO_MAX_REGIONS (same-dtype
        contiguous pairs; any other pair is copied by torch after the batch before it has been
        launched, so a torch copy never overtakes an earlier batched one).  No destination may
        overlap any source or other destination of one batch (the library refuses it)."""
        batch = []

        def flush():
            for k in range(0, len(batch), FVO_MAX_REGIONS):
                part = batch[k:k + FVO_MAX_REGIONS]
                arr = (FvoRegion * len(part))(*[FvoRegion(dp, sp, nb) for dp, sp, nb in part])
                self._check(self.L.fvo_copy_regions(self.h, len(part), ctypes.cast(arr, _P), _stream(self.device)))
            batch.clear()

        for d, src in pairs:
            nb = d.numel() * d.element_size()
            if d.dtype != src.dtype or d.shape != src.shape or not (d.is_contiguous() and src.is_contiguous()):
                flush()
                d.copy_(src)
                continue
            if nb:
                batch.append((d.data_ptr(), src.data_ptr(), nb))
        flush()

    def count_guard(self, counts, n, sets=1, q_counts=None, status=None, code=0, clamped_out=None):
        """fvo_count_guard: status[i] = code where any counts[s*n + i] / q_counts[s*n + i]
        (s < sets) is negative; clamped_out[i] = max(counts[i], 0)."""
        for t in (counts, q_counts, status, clamped_out):
            if t is not None and (t.dtype != torch.int32 or not t.is_contiguous()):
                raise TypeError("count_guard takes contiguous int32 tensors")
        if counts.numel() < sets * n or (q_counts is not None and q_counts.numel() < sets * n):
            raise ValueError("count_guard: counts shorter than sets * n")
        if (status is not None and status.numel() < n) or (clamped_out is not None and clamped_out.numel() < n):
            raise ValueError("count_guard: outputs shorter than n")
        self._check(self.L.fvo_count_guard(self.h, _ptr(counts), _ptr(q_counts), n, sets, _ptr(status), code,
                                           _ptr(clamped_out), _stream(self.device)))

    def voxel_down_sample(self, points, voxel_size, workspace=None):
        """Open3D voxel_down_sample (mono_slam.py:155): points f64 [N,3] (device) ->
        (out f64 [N,3] (first n rows valid, voxel-index order), n i32[1], status i32[1])."""
        if points.dtype != torch.float64 or points.dim() != 2 or points.shape[1] != 3:
            raise TypeError("points must be float64 [N, 3]")
        points = points.contiguous()
        n = points.shape[0]
        out = torch.empty((max(n, 1), 3), dtype=torch.float64, device=self.device)
        cnt = torch.zeros((1,), dtype=torch.int32, device=self.device)
        status = torch.zeros((1,), dtype=torch.int32, device=self.device)
        wb = int(self.L.fvo_voxel_workspace_bytes(n)) if n > 0 else 0
        if n > 0 and wb < 0:
            raise RuntimeError("fvo_voxel_workspace_bytes failed")
        if workspace is None or workspace.numel() < wb:
            workspace = torch.empty((max(wb, 1),), dtype=torch.uint8, device=self.device)
        self._check(self.L.fvo_voxel_down_sample(self.h, _ptr(points), n, float(voxel_size), _ptr(workspace), wb,
                                                 _ptr(out), _ptr(cnt), _ptr(status), _stream(self.device)))
        return out, cnt, status

    def gather_matches(self, kp0, kp1, matches, nmatch, out=None):
        """mkpts0/mkpts1 of a BF match list (fvo_gather_matches): (p0 f32[B,cap,2], p1, n i32[B])."""
        B, cap = matches.shape[0], matches.shape[1]
        if out is None:
            p0 = torch.empty((B, cap, 2), dtype=torch.float32, device=self.device)
            p1 = torch.empty((B, cap, 2), dtype=torch.float32, device=self.device)
            n = torch.empty((B,), dtype=torch.int32, device=self.device)
        else:
            p0, p1, n = out
        self._check(self.L.fvo_gather_matches(self.h, _ptr(kp0), _ptr(kp1), _ptr(matches), _ptr(nmatch), B, cap,
                                              _ptr(p0), _ptr(p1), _ptr(n), _stream(self.device)))
        return p0, p1, n

    def find_essential(self, p0, p1, n, focal, pp, prob=0.999, threshold=1.0, max_iters=1000, out=None):
        """findEssentialMat(RANSAC) on [B] point sets: (E f64[B,3,3], mask u8[B,cap], status i32[B])."""
        B, cap = p0.shape[0], p0.shape[1]
        if out is None:
            E = torch.empty((B, 3, 3), dtype=torch.float64, device=self.device)
            mask = torch.empty((B, cap), dtype=torch.uint8, device=self.device)
            st = torch.empty((B,), dtype=torch.int32, device=self.device)
        else:
            E, mask, st = out
        self._check(self.L.fvo_find_essential(self.h, _ptr(p0.contiguous()), _ptr(p1.contiguous()), _ptr(n), B, cap,
                                              float(focal), float(pp[0]), float(pp[1]), float(prob), float(threshold),
                                              int(max_iters), _ptr(E), _ptr(mask), _ptr(st), _stream(self.device)))
        return E, mask, st

    def recover_pose(self, E, p0, p1, n, focal, pp, e_status=None, distance_thresh=50.0, out=None):
        """recoverPose on [B] frames: (R f64[B,3,3], t f64[B,3], T f64[B,4,4], n_good i32[B])."""
        B, cap = p0.shape[0], p0.shape[1]
        if out is None:
            R = torch.empty((B, 3, 3), dtype=torch.float64, device=self.device)
            t = torch.empty((B, 3), dtype=torch.float64, device=self.device)
            T = torch.empty((B, 4, 4), dtype=torch.float64, device=self.device)
            g = torch.empty((B,), dtype=torch.int32, device=self.device)
        else:
            R, t, T, g = out
        self._check(self.L.fvo_recover_pose(self.h, _ptr(E.contiguous()), _ptr(e_status), _ptr(p0.contiguous()),
                                            _ptr(p1.contiguous()), _ptr(n), B, cap, float(focal), float(pp[0]),
                                            float(pp[1]), float(distance_thresh), _ptr(R), _ptr(t), _ptr(T), _ptr(g),
                                            _stream(self.device)))
        return R, t, T, g

    def debug_buffer(self, which: int) -> torch.Tensor:
        """Host copy (u8 CPU tensor) of an internal workspace buffer (fvo_debug_buffer)."""
        p = ctypes.c_void_p()
        nb = ctypes.c_int64()
        self._check(self.L.fvo_debug_buffer(self.h, which, ctypes.byref(p), ctypes.byref(nb)))
        torch.cuda.synchronize(self.device)
        host = torch.empty((nb.value,), dtype=torch.uint8)
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        if hip.hipMemcpy(ctypes.c_void_p(host.data_ptr()), p, nb.value, 2) != 0:  # 2 = DeviceToHost
            raise RuntimeError("hipMemcpy failed")
        return host

    def geometry(self):
        """Pyramid level (w, h, offset) list, mirroring OpenCV ORB's layer sizes."""
        import numpy as np
        sf = float(np.float32(self.cfg.scale_factor))
        out, off = [], 0
        for l in range(self.cfg.nlevels):
            s = np.float32(sf ** l)
            inv = np.float32(1.0) / s
            w = int(np.rint(np.float32(self.width) * inv))
            h = int(np.rint(np.float32(self.height) * inv))
            out.append((w, h, off))
            off += w * h
        return out, off

    def test_retain_best(self, keys: torch.Tensor, keep: int):
        keys = keys.to(self.device, torch.float32).contiguous()
        n = keys.numel()
        idx = torch.empty((max(n, 1),), dtype=torch.int32, device=self.device)
        nout = torch.empty((1,), dtype=torch.int32, device=self.device)
        self._check(self.L.fvo_test_retain_best(self.h, _ptr(keys), n, keep, _ptr(idx), _ptr(nout),
                                                _stream(self.device)))
        k = int(nout.item())
        return idx[:k].clone()
