"""Map-accumulation kernel throughput: fvo_map_transform on 64 frames x 2000
points (the stereo path's per-frame points3D, stereo_slam.py:308-318) and on one 1M-point cloud
(a lidar-sized map update, mono_slam.py:148), then fvo_voxel_down_sample(0.5) of that cloud
(mono_slam.py:155).  HIP-event times on the launch stream; algorithmic bytes: transform 12 B in +
24 B (f64) + 12 B (f32) out per point; voxel pass 24 B in per point + 24 B per output voxel."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _time(ctx, name, fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ctx.timing_enable([name])
    for _ in range(reps):
        fn()
    ms, n = ctx.timing_read()[name]
    ctx.timing_enable([])
    return ms / n


def main():
    from forest_slam_amd import _lib
    ctx = _lib.Context(64, 64, max_batch=1, stages=_lib.STAGE_BF, kp_capacity=64)
    g = torch.Generator(device="cuda").manual_seed(0)
    T = torch.eye(4, dtype=torch.float64, device="cuda")
    T[:3, 3] = torch.tensor([1.5, -2.0, 0.25])
    for B, cap in [(64, 2000), (1, 1 << 20)]:
        P = torch.randn((B, cap, 3), device="cuda", generator=g) * 20
        n = torch.full((B,), cap, dtype=torch.int32, device="cuda")
        TT = T.expand(B, 4, 4).contiguous()
        m64 = torch.empty((B * cap, 3), dtype=torch.float64, device="cuda")
        m32 = torch.empty((B * cap, 3), dtype=torch.float32, device="cuda")
        cnt = torch.zeros((1,), dtype=torch.int32, device="cuda")

        def run():
            cnt.zero_()
            ctx.map_transform(P, n, TT, cnt, m64, m32)
        ms = _time(ctx, "map_transform", run)
        alg = 48.0 * B * cap
        print(json.dumps({"kernel": "k_map_xform", "sets": B, "points_per_launch": B * cap, "avg_launch_ms": round(ms, 4),
                          "points_per_s": round(B * cap / ms * 1e3, 1), "achieved_gbs": round(alg / ms / 1e6, 1),
                          "peak_gbs": 8000.0, "frac": round(alg / ms / 8e9, 4)}), flush=True)
    cloud = m64[: 1 << 20]
    ws = torch.empty((int(ctx.L.fvo_voxel_workspace_bytes(cloud.shape[0])),), dtype=torch.uint8, device="cuda")
    out = {}

    def vox():
        out["r"] = ctx.voxel_down_sample(cloud, 0.5, workspace=ws)
    ms = _time(ctx, "voxel_down_sample", vox)
    nv = int(out["r"][1].item())
    alg = 24.0 * cloud.shape[0] + 24.0 * nv
    print(json.dumps({"kernel": "voxel_down_sample (bounds+keys+radix sort+scan+average)", "points": cloud.shape[0],
                      "voxels": nv, "avg_ms": round(ms, 4), "points_per_s": round(cloud.shape[0] / ms * 1e3, 1),
                      "achieved_gbs": round(alg / ms / 1e6, 1), "peak_gbs": 8000.0}), flush=True)


if __name__ == "__main__":
    main()
