"""Motion-blur ablation kernel throughput (apply_random_motion_blur,
forest_slam_ros/src/stereo_slam.py:142-178) on a batch of 960x600 gray images resident in HBM,
10 % of the pixels sampled (the function's default; the mask then covers ~all pixels).  HIP-event
time of k_mb_blur on its launch stream -> images/s and GB/s of algorithmic traffic (1 B image
+ 1 B mask read, 1 B written per pixel) against the 8 TB/s HBM peak.  One JSON line per k."""
import json
import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(B=128, W=960, H=600, reps=20, pct=10):
    from forest_slam_amd import _lib
    ctx = _lib.Context(W, H, max_batch=B, stages=_lib.STAGE_BF, kp_capacity=64)
    g = torch.Generator(device="cuda").manual_seed(0)
    img = torch.randint(0, 256, (B, H, W), dtype=torch.uint8, device="cuda", generator=g)
    n = int(H * W * pct / 100)
    C = torch.from_numpy(np.stack([np.asarray(random.Random(b).sample(range(H * W), n), np.int32)
                                   for b in range(B)])).cuda()
    cnt = torch.full((B,), n, dtype=torch.int32, device="cuda")
    out, mask = torch.empty_like(img), torch.empty_like(img)
    for k in (10, 15, 20):
        for _ in range(3):
            ctx.motion_blur(img, k, C, cnt, out=out, mask=mask)
        torch.cuda.synchronize()
        ctx.timing_enable(["motion_blur"])
        for _ in range(reps):
            ctx.motion_blur(img, k, C, cnt, out=out, mask=mask)
        ms, nl = ctx.timing_read()["motion_blur"]
        ctx.timing_enable([])
        per = ms / nl / 1e3
        alg = 3.0 * W * H * B
        print(json.dumps({"kernel": "k_mb_blur", "ksize": k, "path": "direct" if k * k < 130 else "dft-exact",
                          "images_per_launch": B, "mask_coverage": round(float(mask.float().mean()), 4),
                          "avg_launch_ms": round(per * 1e3, 4), "images_per_s": round(B / per, 1),
                          "algorithmic_bytes_per_launch": int(alg), "achieved_gbs": round(alg / per / 1e9, 1),
                          "peak_gbs": 8000.0, "frac": round(alg / per / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
