"""Mono path throughput (BASELINE configs[2]: mono 600p ORB + essential-matrix pose, 1 GPU).
Prints one JSON line: frames/s over B-frame steps, per-kernel ms, and the first step's
RANSAC statistics.  Synthetic forest frames along the 1018_00 path (start=100, moving)."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--width", type=int, default=960)
    ap.add_argument("--height", type=int, default=600)
    ap.add_argument("--interval", type=int, default=1, help="mono_slam.py frame_interval")
    # overlap measured equal (14,836 vs 14,911 frames/s): the essential-matrix stage keeps every SIMD's
    # FP64 issue busy, so ORB beside it gains nothing; in order by default
    ap.add_argument("--overlap", type=int, default=0, help="front stage (ORB + BF) of step k+1 beside step k's back stage")
    a = ap.parse_args()
    from forest_slam_amd import synth, vo
    dev = torch.device("cuda", 0)
    B = a.batch
    seq = synth.StereoSequence(seed=0, n_frames=(B + 1) * a.interval, W=a.width, H=a.height, device=dev, start=100)
    L, _ = seq.frames(range(0, (B + 1) * a.interval, a.interval))
    fe = vo.MonoFrontEnd(a.width, a.height, seq.K, batch=B, nfeatures=a.nfeatures, device=dev, overlap=bool(a.overlap))
    fe.prime(L[0])
    Lb = L[1:].contiguous()
    for _ in range(a.warmup):
        fe.step(Lb)
    torch.cuda.synchronize()
    fe.ctx.timing_enable(None)
    fe.step(Lb)
    stages = {k: round(v[0], 4) for k, v in sorted(fe.ctx.timing_read().items(), key=lambda kv: -kv[1][0])}
    fe.ctx.timing_enable([])
    st = fe.status[:B].cpu()
    ng = fe.ngood[:B].cpu()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        fe.step(Lb)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"metric": "mono frames/sec (ORB + BF + findEssentialMat + recoverPose)", "value":
                      round(B * a.steps / el, 2), "unit": "frames/s", "ms_per_step": round(el / a.steps * 1e3, 3),
                      "config": {"workload": "configs[2] mono", "width": a.width, "height": a.height,
                                 "nfeatures": a.nfeatures, "frames_per_step": B, "overlap": bool(a.overlap)},
                      "stages_ms_per_step": stages, "status_ok": int((st == 1).sum()),
                      "mean_cheirality_inliers": float(ng[st == 1].float().mean()) if (st == 1).any() else None}))


if __name__ == "__main__":
    main()
