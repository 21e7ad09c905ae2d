"""Ingest kernel throughput (cv2.undistort + BGR2GRAY, stereo_slam.py:184-186)
on a batch of 960x600 BGR8 images resident in HBM; HIP-event time of the kernel on its launch
stream -> images/s and GB/s of algorithmic traffic (3 B read + 1 B written per pixel) against
the 8 TB/s HBM peak.  Prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
K0 = np.array([[642.9165664800531, 0., 460.1840658156501], [0., 641.9171825800378, 308.5846449100310], [0., 0., 1.]])
DIST_L = np.array([-0.060164620903866, 0.094005180631043, 0.0, 0.0, 0])


def main(B=128, W=960, H=600, reps=20):
    from forest_slam_amd import _lib
    ctx = _lib.Context(W, H, max_batch=B, stages=_lib.STAGE_ORB)
    g = torch.Generator(device="cuda").manual_seed(0)
    bgr = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        ctx.undistort_gray(bgr, K0, DIST_L, out=out)
    torch.cuda.synchronize()
    ctx.timing_enable(["ingest_undistort_gray"])
    for _ in range(reps):
        ctx.undistort_gray(bgr, K0, DIST_L, out=out)
    ms, n = ctx.timing_read()["ingest_undistort_gray"]
    ctx.timing_enable([])
    per = ms / n / 1e3
    alg = 4.0 * W * H * B
    print(json.dumps({"kernel": "k_ing_undistort_gray", "images_per_launch": B, "avg_launch_ms": round(per * 1e3, 4),
                      "images_per_s": round(B / per, 1), "algorithmic_bytes_per_launch": int(alg),
                      "achieved_gbs": round(alg / per / 1e9, 1), "peak_gbs": 8000.0,
                      "frac": round(alg / per / 8e12, 4)}))


if __name__ == "__main__":
    main()
