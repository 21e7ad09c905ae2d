"""Overlapped 600p step with the front stage (SGBM + ORB + BF) on a CU-masked stream, so a few CUs
stay free for the back stage's dispatches (tooling experiment: prints frames/s per mask).

    python tools/bench_cumask.py [--masks none,lo16,stride16] [--steps 10]

lo16 masks out CUs 0..15, stride16 every 16th CU (which of the two spreads the reserved CUs
over the 8 XCDs depends on the driver's CU numbering, hence both); hiprio puts the back stage,
fronthi the front stage on a high-priority stream."""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def masked_stream(dev, kind):
    if kind in ("none", "hiprio"):
        return torch.cuda.Stream(dev)
    if kind == "fronthi":  # the front stage (the step's critical path) on a high-priority stream
        return torch.cuda.Stream(dev, priority=-1)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = [0] * ((ncu + 31) // 32)
    for cu in range(ncu):
        off = (cu < 16) if kind == "lo16" else (cu % 16 == 0) if kind == "stride16" else (cu % 32 == 0)
        if not off:
            words[cu // 32] |= 1 << (cu % 32)
    hip = ctypes.CDLL("libamdhip64.so")
    s = ctypes.c_void_p()
    arr = (ctypes.c_uint32 * len(words))(*words)
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return torch.cuda.ExternalStream(s.value, device=dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--masks", default="none,hiprio,lo16,stride16,stride32,none")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    from forest_slam_amd import synth, vo
    dev = torch.device("cuda", 0)
    B, W, H = 64, 960, 600
    seq = synth.StereoSequence(seed=0, n_frames=B + 1, W=W, H=H, device=dev)
    L, R = seq.frames(range(B + 1))
    Lb, Rb = L[1:].contiguous(), R[1:].contiguous()
    for kind in a.masks.split(","):
        fe = vo.StereoFrontEnd(W, H, seq.K, synth.DIST_L, synth.BASELINE, batch=B, nfeatures=1000, device=dev,
                               ba_window=10, overlap_sgbm=True)
        fe.s_sgbm = masked_stream(dev, kind)
        # hiprio: the back stage (the caller's stream) on a high-priority stream
        main = torch.cuda.Stream(dev, priority=-1) if kind == "hiprio" else torch.cuda.current_stream(dev)
        with torch.cuda.stream(main):
            fe.prime(L[0], R[0])
            for _ in range(3):
                fe.step(Lb, Rb)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                fe.step(Lb, Rb)
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        print(json.dumps({"mask": kind, "ms_per_step": round(dt * 1e3, 3), "frames_per_s": round(B / dt, 1)}), flush=True)
        del fe
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
