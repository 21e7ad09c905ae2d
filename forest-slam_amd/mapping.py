"""Map accumulation on the GPU over libfvo's fvo_map_transform and
fvo_voxel_down_sample.

* ``PointMap.add_frames`` — stereo_slam.py:308-318: every frame's points3D transformed by its
  cumulative pose, ``(cum @ hstack(points3D, 1).T)[:3].T``, appended to ``all_points_3D``;
  ``cloud32()`` is the float32 x/y/z payload ``create_point_cloud(np.concatenate(...))`` packs
  (PointCloud2, point_step 12).
* ``PointMap.add_cloud`` — mono_slam.py:144-164 / gt_mapping.py:62-66: one point cloud
  transformed by the pose, ``voxel_down_sample(voxel_size=0.5)``, appended to the map.

The map lives in HBM (fp64 + the float32 record), sized once; the append offset is a device
counter, so batches append without host synchronisation."""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


class PointMap:
    def __init__(self, capacity: int, device="cuda:0", ctx: _lib.Context | None = None):
        self.dev = torch.device(device)
        self.ctx = ctx or _lib.Context(64, 64, max_batch=1, stages=_lib.STAGE_BF, kp_capacity=64, device=self.dev)
        self.capacity = int(capacity)
        self.xyz64 = torch.zeros((self.capacity, 3), dtype=torch.float64, device=self.dev)
        self.xyz32 = torch.zeros((self.capacity, 3), dtype=torch.float32, device=self.dev)
        self.count = torch.zeros((1,), dtype=torch.int32, device=self.dev)
        self._tmp64 = None
        self._ws = None

    def __len__(self) -> int:
        n = int(self.count.item())
        if n > self.capacity:
            raise RuntimeError(f"PointMap overflow: {n} points for capacity {self.capacity}")
        return n

    def add_frames(self, points: torch.Tensor, n_points: torch.Tensor, cum: np.ndarray | torch.Tensor,
                   check: bool = False):
        """points f32 [B,cap,3] (device), n_points i32 [B] (device; 0 for frames the reference
        skips), cum f64 [B,4,4] (each frame's cumulative pose, stereo_slam.py:306).

        The device counter keeps counting points past ``capacity`` (they are not written), so
        an overflow is detected exactly by the next ``len()``; ``check=True`` synchronises
        and raises right here instead, before another batch is appended."""
        T = torch.as_tensor(np.asarray(cum, np.float64) if not isinstance(cum, torch.Tensor) else cum,
                            dtype=torch.float64).to(self.dev)
        self.ctx.map_transform(points, n_points, T, self.count, self.xyz64, self.xyz32)
        if check:
            len(self)

    def overflowed(self) -> bool:
        """True once more points were appended than the map holds (host sync)."""
        return int(self.count.item()) > self.capacity

    def add_cloud(self, points, cum, voxel_size: float = 0.5):
        """mono_slam.py:144-164: points f32 [n,3] (PointCloud2 x/y/z), pose cum f64 [4,4]."""
        P = torch.as_tensor(np.asarray(points, np.float32) if not isinstance(points, torch.Tensor) else points,
                            dtype=torch.float32).to(self.dev).reshape(1, -1, 3).contiguous()
        n = P.shape[1]
        if n == 0:
            return
        if self._tmp64 is None or self._tmp64.shape[0] < n:
            self._tmp64 = torch.empty((n, 3), dtype=torch.float64, device=self.dev)
            self._ws = torch.empty((int(self.ctx.L.fvo_voxel_workspace_bytes(n)),), dtype=torch.uint8,
                                   device=self.dev)
        c0 = torch.zeros((1,), dtype=torch.int32, device=self.dev)
        T = torch.as_tensor(np.asarray(cum, np.float64), dtype=torch.float64, device=self.dev).reshape(1, 4, 4)
        self.ctx.map_transform(P, torch.tensor([n], dtype=torch.int32, device=self.dev), T, c0, self._tmp64[:n], None)
        out, nv, st = self.ctx.voxel_down_sample(self._tmp64[:n], voxel_size, workspace=self._ws)
        if int(st.item()) != 0:
            raise RuntimeError("voxel_down_sample: voxel index outside the 21-bit key range")
        k, base = int(nv.item()), len(self)
        if base + k > self.capacity:
            raise RuntimeError(f"PointMap overflow: {base + k} points for capacity {self.capacity}")
        self.xyz64[base:base + k] = out[:k]
        self.xyz32[base:base + k] = out[:k].to(torch.float32)  # pc2.create_cloud_xyz32
        self.count += k

    def cloud32(self) -> np.ndarray:
        return self.xyz32[: len(self)].cpu().numpy()

    def cloud64(self) -> np.ndarray:
        return self.xyz64[: len(self)].cpu().numpy()
