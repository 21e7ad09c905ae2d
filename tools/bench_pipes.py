"""Throughput of P independent front-end pipelines sharing one GPU (experiment tool).

Each pipeline is its own StereoFrontEnd (own context, own HIP streams) fed from its own
caller stream; all are enqueued back to back every step, so the hardware interleaves their
kernels freely.  Comparing P = 1 and P = 2 frames/s tells how much of one pipeline's step is
latency the GPU could fill with other work (the upper bound of any stream re-arrangement
inside one pipeline).

    python tools/bench_pipes.py --pipes 2 --steps 10 [--overlap-sgbm 1]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pipes", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--overlap-sgbm", type=int, default=1)
    a = ap.parse_args()
    from forest_slam_amd import synth, vo
    B = a.batch
    seq = synth.StereoSequence(seed=0, n_frames=B + 1, W=960, H=600, device="cuda")
    L, R = seq.frames(range(B + 1))
    fwd = (L[1:].contiguous(), R[1:].contiguous())
    bwd = (L[:B].flip(0).contiguous(), R[:B].flip(0).contiguous())
    pipes = []
    for _ in range(a.pipes):
        fe = vo.StereoFrontEnd(960, 600, seq.K, synth.DIST_L, synth.BASELINE, batch=B, nfeatures=1000, ba_window=10,
                               overlap_sgbm=bool(a.overlap_sgbm))
        fe.prime(L[0], R[0])
        pipes.append((fe, torch.cuda.Stream()))
    n = [0]

    def step():
        src = fwd if n[0] % 2 == 0 else bwd
        n[0] += 1
        for fe, s in pipes:
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fe.step(*src)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"pipes": a.pipes, "frames_per_s": round(a.pipes * B * a.steps / dt, 1),
                      "ms_per_step": round(dt / a.steps * 1e3, 3), "overlap_sgbm": a.overlap_sgbm}))


if __name__ == "__main__":
    main()
