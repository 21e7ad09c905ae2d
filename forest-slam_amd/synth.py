"""Synthetic rectified forest stereo sequences (SURVEY.md §8d workload).

Test/bench input generator, not part of the measured path.  The reference runs on the
BotanicGarden 1018_00 rosbag (``stereo_slam.py:35``), which does not exist in this
container or on the GPU box, so frames are ray-cast here instead:

* camera: K0 of ``stereo_slam.py:45-47``; right camera shifted by the baseline the
  reference actually uses, ``np.linalg.norm(T_rgb0_rgb1[:3, 3])`` evaluated on the
  (1,16)-shaped array = 0.253736175410149 m (``stereo_slam.py:61-64,270``);
* path: the 1018_00 ground-truth positions (963 poses, 10 Hz, y is down), heading from
  the direction of travel;
* scene (seed ``s``): vertical trunks with multi-octave value-noise bark, a textured
  ground plane, sky; Gaussian sensor noise sigma 2 DN, clamped to u8.

Everything is plain torch so it runs on the GPU box's device or on the CPU for tests.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

K0 = np.array([[642.9165664800531, 0.0, 460.1840658156501],
               [0.0, 641.9171825800378, 308.5846449100310],
               [0.0, 0.0, 1.0]])
DIST_L = np.array([-0.060164620903866, 0.094005180631043, 0.0, 0.0, 0.0])
BASELINE = 0.253736175410149
_GT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "1018_00_Ground_Truth.txt")


def load_tum(path: str) -> np.ndarray:
    return np.loadtxt(path, dtype=np.float64).reshape(-1, 8)


def gt_path(n: int | None = None, stride: int = 1) -> tuple[np.ndarray, np.ndarray]:
    """Returns (timestamps f64[n], camera-to-world f64[n,4,4]) along the 1018_00 path."""
    gt = load_tum(_GT)
    t, p = gt[:, 0], gt[:, 1:4].copy()
    # heading from the displacement over +-1.5 s in the horizontal (x, z) plane; y is down.
    # While the vehicle (nearly) stands still the GT jitter would make that direction
    # spin, so the heading is held: frames whose 3 s displacement is under 0.3 m keep the
    # previous heading (the first moving heading for a stationary start).
    k = 15
    pad = np.pad(p, ((k, k), (0, 0)), mode="edge")
    fwd = pad[2 * k:] - pad[:-2 * k]
    fwd[:, 1] = 0.0
    nrm = np.linalg.norm(fwd, axis=1, keepdims=True)
    moving = nrm[:, 0] > 0.3
    fwd = np.where(moving[:, None], fwd / np.maximum(nrm, 1e-12), np.array([0.0, 0.0, 1.0]))
    if moving.any():
        first = int(np.argmax(moving))
        fwd[:first] = fwd[first]
    for i in range(1, len(fwd)):
        if not moving[i]:
            fwd[i] = fwd[i - 1]
    down = np.array([0.0, 1.0, 0.0])
    T = np.zeros((len(p), 4, 4))
    for i in range(len(p)):
        z = fwd[i]
        x = np.cross(down, z)
        x /= np.linalg.norm(x)
        y = np.cross(z, x)
        T[i, :3, :3] = np.stack([x, y, z], 1)
        T[i, :3, 3] = p[i]
        T[i, 3, 3] = 1.0
    sel = slice(0, None if n is None else n * stride, stride)
    return t[sel], T[sel]


def _hash2(ix: torch.Tensor, iy: torch.Tensor, seed: int) -> torch.Tensor:
    h = (ix * 374761393 + iy * 668265263 + seed * 2147483647) & 0xFFFFFFFF
    h = ((h ^ (h >> 13)) * 1274126177) & 0xFFFFFFFF
    h = h ^ (h >> 16)
    return (h & 0xFFFF).to(torch.float32) / 65535.0


def value_noise(x: torch.Tensor, y: torch.Tensor, seed: int) -> torch.Tensor:
    x0, y0 = torch.floor(x), torch.floor(y)
    fx, fy = x - x0, y - y0
    ix, iy = x0.to(torch.int64), y0.to(torch.int64)
    sx, sy = fx * fx * (3 - 2 * fx), fy * fy * (3 - 2 * fy)
    a = _hash2(ix, iy, seed)
    b = _hash2(ix + 1, iy, seed)
    c = _hash2(ix, iy + 1, seed)
    d = _hash2(ix + 1, iy + 1, seed)
    return (a + (b - a) * sx) + ((c + (d - c) * sx) - (a + (b - a) * sx)) * sy


def fbm(x: torch.Tensor, y: torch.Tensor, seed: int, octaves: int = 5) -> torch.Tensor:
    out = torch.zeros_like(x)
    amp, tot = 1.0, 0.0
    for o in range(octaves):
        out = out + amp * value_noise(x, y, seed + 17 * o)
        tot += amp
        x, y = x * 2.03, y * 2.03
        amp *= 0.55
    return out / tot


class ForestScene:
    """Trunks (cx, cz, r) placed around a camera path; seed picks the forest."""

    def __init__(self, path_T: np.ndarray, seed: int = 0, n_trees: int = 400, margin: float = 15.0,
                 corridor: float = 2.0, ground_drop: float = 1.5):
        rng = np.random.default_rng(seed)
        p = path_T[:, :3, 3]
        lo = p[:, [0, 2]].min(0) - margin
        hi = p[:, [0, 2]].max(0) + margin
        trees = []
        tries = 0
        while len(trees) < n_trees and tries < n_trees * 50:
            tries += 1
            c = rng.uniform(lo, hi)
            r = rng.uniform(0.15, 0.5)
            dmin = np.min(np.hypot(p[:, 0] - c[0], p[:, 2] - c[1]))
            if dmin < corridor + r:
                continue
            trees.append((c[0], c[1], r))
        self.trees = np.array(trees, dtype=np.float64)
        self.ground_y = float(p[:, 1].max() + ground_drop)
        self.seed = seed


@torch.no_grad()
def render(scene: ForestScene, T_wc: np.ndarray, K: np.ndarray, W: int, H: int, device="cpu",
           noise_seed: int | None = None, max_dist: float = 60.0, chunk: int = 1 << 15) -> torch.Tensor:
    """Render one u8[H,W] grayscale view from camera-to-world T_wc."""
    dev = torch.device(device)
    f32 = torch.float32
    R = torch.tensor(T_wc[:3, :3], dtype=f32, device=dev)
    o = torch.tensor(T_wc[:3, 3], dtype=f32, device=dev)
    vv, uu = torch.meshgrid(torch.arange(H, device=dev, dtype=f32), torch.arange(W, device=dev, dtype=f32),
                            indexing="ij")
    dc = torch.stack([(uu - K[0, 2]) / K[0, 0], (vv - K[1, 2]) / K[1, 1], torch.ones_like(uu)], -1).reshape(-1, 3)
    d = dc @ R.T
    n = d.shape[0]
    # cull trees to those near the camera
    tr = scene.trees
    near = np.hypot(tr[:, 0] - T_wc[0, 3], tr[:, 1] - T_wc[2, 3]) < max_dist
    trees = torch.tensor(tr[near], dtype=f32, device=dev)
    best = torch.full((n,), float("inf"), device=dev)
    tid = torch.full((n,), -1, dtype=torch.int64, device=dev)
    dxz = d[:, [0, 2]]
    a = (dxz * dxz).sum(1).clamp_min(1e-12)
    oc = o[[0, 2]]
    for s in range(0, trees.shape[0], 64):
        tt = trees[s:s + 64]
        for c0 in range(0, n, chunk):
            dd, aa = dxz[c0:c0 + chunk], a[c0:c0 + chunk]
            m = oc[None, :] - tt[:, :2]                             # [T,2]
            b = dd @ m.T                                           # [N,T]
            cc = (m * m).sum(1)[None, :] - tt[:, 2][None, :] ** 2  # [1,T]
            disc = b * b - aa[:, None] * cc
            s_hit = (-b - torch.sqrt(disc.clamp_min(0))) / aa[:, None]
            s_hit = torch.where((disc > 0) & (s_hit > 0.05), s_hit, torch.full_like(s_hit, float("inf")))
            v, idx = s_hit.min(1)
            upd = v < best[c0:c0 + chunk]
            best[c0:c0 + chunk] = torch.where(upd, v, best[c0:c0 + chunk])
            tid[c0:c0 + chunk] = torch.where(upd, idx + s, tid[c0:c0 + chunk])
    # ground plane (y down): hit when ray goes down
    sg = torch.where(d[:, 1] > 1e-6, (scene.ground_y - o[1]) / d[:, 1].clamp_min(1e-6),
                     torch.full((n,), float("inf"), device=dev))
    ground = sg < best
    s_fin = torch.where(ground, sg, best)
    p = o[None, :] + s_fin[:, None].clamp(max=1e4) * d
    val = torch.full((n,), 0.85, device=dev)  # sky
    seed = scene.seed * 7919
    # bark
    hit_t = (tid >= 0) & ~ground & torch.isfinite(best)
    if hit_t.any():
        t = trees[tid.clamp_min(0)]
        ang = torch.atan2(p[:, 2] - t[:, 1], p[:, 0] - t[:, 0])
        arc = ang * t[:, 2]
        tex = fbm(arc * 9.0 + tid.to(f32) * 13.7, p[:, 1] * 3.0, seed + 1)
        fine = fbm(arc * 40.0, p[:, 1] * 10.0, seed + 5, 3) - 0.5
        furrow = (value_noise(arc * 25.0, p[:, 1] * 1.5, seed + 11) > 0.72).to(f32)
        tex = (0.5 + 1.8 * (tex - 0.5) + 0.9 * fine - 0.35 * furrow).clamp(0.02, 1.0)
        shade = 0.55 + 0.45 * torch.cos(ang - 0.7).clamp_min(0)
        val = torch.where(hit_t, tex * shade, val)
    hit_g = ground & torch.isfinite(sg)
    if hit_g.any():
        tex = fbm(p[:, 0] * 2.5, p[:, 2] * 2.5, seed + 3)
        fine = fbm(p[:, 0] * 11.0, p[:, 2] * 11.0, seed + 9, 3) - 0.5
        tex = (0.45 + 1.5 * (tex - 0.5) + 1.0 * fine).clamp(0.02, 1.0)
        val = torch.where(hit_g, tex, val)
    dist = torch.where(hit_t | hit_g, s_fin, torch.full_like(s_fin, max_dist))
    fog = torch.exp(-dist / 45.0)
    val = val * fog + 0.7 * (1 - fog)
    img = val.reshape(H, W) * 255.0
    if noise_seed is not None:
        g = torch.Generator(device="cpu").manual_seed(int(noise_seed))
        img = img + 2.0 * torch.randn(H, W, generator=g).to(dev)
    return img.round().clamp(0, 255).to(torch.uint8)


def scaled_K(W: int, H: int) -> np.ndarray:
    """K0 for 960x600; scaled (fx*s, cx*s) for other sizes."""
    s = W / 960.0
    K = K0.copy()
    K[0, :] *= s
    K[1, :] *= H / 600.0
    return K


class StereoSequence:
    """Rectified synthetic stereo sequence along the 1018_00 path."""

    def __init__(self, seed: int = 0, n_frames: int = 963, W: int = 960, H: int = 600, device="cpu",
                 stride: int = 1, n_trees: int = 400, start: int = 0):
        t, T_wc = gt_path(start + n_frames, stride)
        self.t, self.T_wc = t[start:], T_wc[start:]
        self.n = len(self.t)
        self.W, self.H = W, H
        self.K = scaled_K(W, H)
        self.seed = seed
        self.scene = ForestScene(self.T_wc, seed=seed, n_trees=n_trees)
        self.device = device
        off = np.eye(4)
        off[0, 3] = BASELINE
        self._right = off

    def frame(self, i: int):
        Tl = self.T_wc[i]
        Tr = Tl @ self._right
        L = render(self.scene, Tl, self.K, self.W, self.H, self.device, noise_seed=self.seed * 100003 + 2 * i + 1000)
        R = render(self.scene, Tr, self.K, self.W, self.H, self.device, noise_seed=self.seed * 100003 + 2 * i + 1001)
        return L, R

    def frames(self, idx):
        Ls, Rs = [], []
        for i in idx:
            L, R = self.frame(i)
            Ls.append(L)
            Rs.append(R)
        return torch.stack(Ls), torch.stack(Rs)
