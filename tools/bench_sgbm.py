#!/usr/bin/env python3
"""SGBM alone on the GPU: B=64 synthetic 960x600 pairs, per-kernel times (HIP events) and
the whole-call time, for the schedule / cost-pass launch shape given on the command line
(fvo_config.sgbm_mode / sgbm_lanes / sgbm_cols):
    python tools/bench_sgbm.py [--mode classic|lpath] [--lanes G] [--cols CB] [--batch B]
Prints one JSON line."""
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
    ap.add_argument("--mode", choices=["classic", "lpath"], default="classic")
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--cols", type=int, default=0)
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    from forest_slam_amd import _lib, synth
    B, W, H = a.batch, 960, 600
    seq = synth.StereoSequence(seed=0, n_frames=B, W=W, H=H, device="cuda")
    L, R = seq.frames(range(B))
    mode = _lib.SGBM_LPATH if a.mode == "lpath" else _lib.SGBM_CLASSIC
    ctx = _lib.Context(W, H, max_batch=B, stages=_lib.STAGE_SGBM, sgbm_mode=mode, sgbm_lanes=a.lanes,
                       sgbm_cols=a.cols)
    out = torch.empty((B, H, W), dtype=torch.int16, device="cuda")
    for _ in range(2):
        ctx.sgbm(L, R, out=out)
    torch.cuda.synchronize()
    n = 5
    t0 = time.perf_counter()
    for _ in range(n):
        ctx.sgbm(L, R, out=out)
    torch.cuda.synchronize()
    call_ms = (time.perf_counter() - t0) / n * 1e3
    ctx.timing_enable(None)
    for _ in range(n):
        ctx.sgbm(L, R, out=out)
    torch.cuda.synchronize()
    st = {k: round(v[0] / n, 4) for k, v in ctx.timing_read().items()}
    ctx.timing_enable([])
    var = {"mode": a.mode, "lanes": a.lanes, "cols": a.cols}
    print(json.dumps({"variant": var, "call_ms": round(call_ms, 3), "kernels_ms": st,
                      "workspace_gb": round(ctx.workspace_bytes / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
