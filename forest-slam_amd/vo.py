"""Batched stereo-VO front end on the GPU — the ORB branch of ros_ws/src/stereo_slam.py.

One ``StereoFrontEnd.step`` processes B consecutive stereo frames of one sequence in a
fixed sequence of HIP launches (no host synchronisation inside):

  ORB on the B current left + B current right images          (stereo_slam.py:232-233,240-241)
  BF cross-check match prev->cur, left and right (right unused,
  kept for work-equivalence with the reference)                (:234,242)
  SGBM of the B *previous* stereo pairs                         (:262 -> :108-117)
  back-projection of the matched previous-left keypoints        (:265-289)
  PnP-RANSAC + Rodrigues -> relative T                          (:292-303)

Frames of a sequence are independent except through the chained pose (:306), which the
host composes left to right in float64 (``eval.chain``), so batching B frames per step is
exact.  The previous image / keypoints of the last frame are carried to
the next step.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


class StereoFrontEnd:
    def __init__(self, width: int, height: int, K: np.ndarray, dist: np.ndarray, baseline: float, batch: int,
                 nfeatures: int = 500, match_right: bool = True, device=None, **params):
        self.B = batch
        self.K = np.asarray(K, np.float64)
        self.dist = np.resize(np.asarray(dist, np.float64), 5)
        self.baseline = float(baseline)
        self.match_right = match_right
        self.ctx = _lib.Context(width, height, max_batch=2 * batch, device=device, nfeatures=nfeatures, **params)
        self.dev = self.ctx.device
        self.cap = self.ctx.kp_cap
        self.W, self.H = width, height
        B, cap, dev = batch, self.cap, self.dev
        e = lambda shape, dt: torch.empty(shape, dtype=dt, device=dev)  # noqa: E731
        # persistent device buffers (no allocation inside step)
        self.kp = e((2 * B, cap, _lib.KP_STRIDE), torch.float32)
        self.desc = e((2 * B, cap, _lib.DESC_BYTES), torch.uint8)
        self.cnt = e((2 * B,), torch.int32)
        self.q_desc = e((2 * B, cap, _lib.DESC_BYTES), torch.uint8)
        self.q_cnt = e((2 * B,), torch.int32)
        self.q_kp = e((B, cap, _lib.KP_STRIDE), torch.float32)
        self.matches = e((2 * B, cap, 3), torch.int32)
        self.nmatch = e((2 * B,), torch.int32)
        self.prevL = e((B, height, width), torch.uint8)
        self.prevR = e((B, height, width), torch.uint8)
        self.disp = e((B, height, width), torch.int16)
        self.P3 = e((B, cap, 3), torch.float32)
        self.p2 = e((B, cap, 2), torch.float32)
        self.npts = e((B,), torch.int32)
        self.rvec = e((B, 3), torch.float64)
        self.tvec = e((B, 3), torch.float64)
        self.T = e((B, 4, 4), torch.float64)
        self.status = e((B,), torch.int32)
        self.inl = e((B, cap), torch.uint8)
        self.imgs = e((2 * B, height, width), torch.uint8)
        self.has_prev = False
        self.last = None  # (L, R, kpL, descL, cntL, descR, cntR) of the last processed image pair

    def prime(self, L0: torch.Tensor, R0: torch.Tensor):
        """Feed the first stereo pair of a sequence (no pose is produced for it)."""
        imgs = torch.stack([L0, R0]).to(self.dev)
        kp, desc, cnt = self.ctx.orb(imgs)
        self.last = (imgs[0].clone(), imgs[1].clone(), kp[0].clone(), desc[0].clone(), cnt[0:1].clone(),
                     desc[1].clone(), cnt[1:2].clone())
        self.has_prev = True

    def step(self, L: torch.Tensor, R: torch.Tensor):
        """L, R: u8 [n,H,W] device tensors, n <= B consecutive frames after the primed/last
        pair.  Returns (T_rel f64[n,4,4], status i32[n]) device tensors (async)."""
        if not self.has_prev:
            raise RuntimeError("call prime() with the first stereo pair first")
        n = L.shape[0]
        B = self.B
        if n > B:
            raise ValueError("more frames than the configured batch")
        ctx = self.ctx
        self.imgs[:n].copy_(L)
        self.imgs[n:2 * n].copy_(R)
        kp, desc, cnt = ctx.orb(self.imgs[:2 * n], out=(self.kp[:2 * n], self.desc[:2 * n], self.cnt[:2 * n]))
        lastL, lastR, lkp, ldesc, lcnt, rdesc, rcnt = self.last
        # query (previous) descriptor sets: left frames then right frames
        self.q_desc[0].copy_(ldesc)
        self.q_cnt[0:1].copy_(lcnt)
        if n > 1:
            self.q_desc[1:n].copy_(desc[:n - 1])
            self.q_cnt[1:n].copy_(cnt[:n - 1])
        self.q_desc[n].copy_(rdesc)
        self.q_cnt[n:n + 1].copy_(rcnt)
        if n > 1:
            self.q_desc[n + 1:2 * n].copy_(desc[n:2 * n - 1])
            self.q_cnt[n + 1:2 * n].copy_(cnt[n:2 * n - 1])
        nb = 2 * n if self.match_right else n
        m, nm = ctx.bf_match(self.q_desc[:nb], self.q_cnt[:nb], desc[:nb], cnt[:nb],
                             out=(self.matches[:nb], self.nmatch[:nb]))
        # previous stereo pairs for SGBM and previous-left keypoints for back-projection
        self.prevL[0].copy_(lastL)
        self.prevR[0].copy_(lastR)
        self.q_kp[0].copy_(lkp)
        if n > 1:
            self.prevL[1:n].copy_(L[:n - 1])
            self.prevR[1:n].copy_(R[:n - 1])
            self.q_kp[1:n].copy_(kp[:n - 1])
        disp = ctx.sgbm(self.prevL[:n], self.prevR[:n], out=self.disp[:n])
        P3, p2, npts = ctx.backproject(disp, self.q_kp[:n], kp[:n], m[:n], nm[:n], self.K, self.baseline,
                                       out=(self.P3[:n], self.p2[:n], self.npts[:n]))
        rv, tv, T, st, _ = ctx.pnp_ransac(P3, p2, npts, self.K, self.dist,
                                          out=(self.rvec[:n], self.tvec[:n], self.T[:n], self.status[:n],
                                               self.inl[:n]))
        self.last = (L[n - 1].clone(), R[n - 1].clone(), kp[n - 1].clone(), desc[n - 1].clone(),
                     cnt[n - 1:n].clone(), desc[2 * n - 1].clone(), cnt[2 * n - 1:2 * n].clone())
        return T, st


def run_sequence(frontend: StereoFrontEnd, L_all: torch.Tensor, R_all: torch.Tensor, stamps=None):
    """Process a whole sequence (images on device) -> (TUM rows, relative poses, statuses)."""
    from . import eval as ev
    n = L_all.shape[0]
    frontend.prime(L_all[0], R_all[0])
    Ts, sts = [], []
    for s in range(1, n, frontend.B):
        e = min(s + frontend.B, n)
        T, st = frontend.step(L_all[s:e], R_all[s:e])
        Ts.append(T.cpu().numpy())
        sts.append(st.cpu().numpy())
    T = np.concatenate(Ts) if Ts else np.zeros((0, 4, 4))
    st = np.concatenate(sts) if sts else np.zeros((0,), np.int32)
    # status -1 = fewer than 6 points: the reference skips the frame (no pose, no TUM row,
    # stereo_slam.py:292); status 0 = RANSAC failure: identity T (the reference would chain
    # whatever solvePnPRansac left in rvec/tvec), row emitted.
    valid = st != -1
    cum = ev.chain(T, valid)
    if stamps is None:
        stamps = np.arange(n, dtype=np.float64)
    rows = ev.tum_rows(np.asarray(stamps)[1:][valid], cum)
    return rows, T, st
