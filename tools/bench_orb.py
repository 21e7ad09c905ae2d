#!/usr/bin/env python3
"""ORB alone on the GPU (tooling): the bench step's ORB call -- 64 left + 64 right synthetic
960x600 images, nfeatures 1000 -- with per-kernel times (HIP events) and the whole-call time.
Prints one JSON line; FVO_LIB selects a variant library."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from forest_slam_amd import _lib, synth
    B, W, H = 64, 960, 600
    seq = synth.StereoSequence(seed=0, n_frames=B, W=W, H=H, device="cuda")
    L, R = seq.frames(range(B))
    imgs = torch.cat([L, R]).contiguous()
    ctx = _lib.Context(W, H, max_batch=2 * B, nfeatures=1000, stages=_lib.STAGE_ORB)
    out = None
    for _ in range(2):
        out = ctx.orb(imgs)
    torch.cuda.synchronize()
    n = 5
    t0 = time.perf_counter()
    for _ in range(n):
        out = ctx.orb(imgs)
    torch.cuda.synchronize()
    call_ms = (time.perf_counter() - t0) / n * 1e3
    ctx.timing_enable(None)
    for _ in range(n):
        ctx.orb(imgs)
    torch.cuda.synchronize()
    st = {k: round(v[0] / n, 4) for k, v in ctx.timing_read().items()}
    ctx.timing_enable([])
    counts = out[2].cpu()
    print(json.dumps({"call_ms": round(call_ms, 3), "kernels_ms": st, "kp_checksum": int(counts.sum())}), flush=True)


if __name__ == "__main__":
    main()
