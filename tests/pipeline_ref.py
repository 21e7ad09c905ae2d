"""Oracle-side pipeline of stereo_slam.py's ORB branch (:232-306) plus the local-BA
specification, over a whole frame sequence — the checker of the end-to-end GPU tests.

Test infrastructure only.  Frame pairs are independent, so the oracle work
is spread over a thread pool (the oracle's ctypes calls release the GIL)."""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np


def threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def sequence(oracle_mod, frames, K, dist, baseline, nfeatures):
    """frames: list of (L, R) u8 arrays.  Returns (pairs, kps): pairs[j] = oracle.frame_pose of
    (frames[j], frames[j+1]) (matches, disp16, P3, T, ...), kps[j] = the left keypoints of frame j."""
    n = len(frames)
    with ThreadPoolExecutor(max_workers=threads()) as ex:
        pairs = list(ex.map(lambda j: oracle_mod.frame_pose(frames[j][0], frames[j][1], frames[j + 1][0], K, dist,
                                                            baseline, nfeatures), range(n - 1)))
    kps = [p["kp0"] for p in pairs] + [pairs[-1]["kp1"]]
    return pairs, kps


def ba_windows(ba_ref, pairs, kps, rel, K, baseline, window, ends, iters=10):
    """ba_ref.ba_window for every window end e in `ends` (frames max(0, e-K+1) .. e), with the
    relative transforms `rel` (camera j -> j+1) as the initial poses.  Returns {e: ref}
    (None for windows of fewer than 3 frames, which pass the PnP transform through)."""
    stereo = [ba_ref.stereo_points(kps[j], pairs[j]["disp16"], K, baseline) for j in range(len(pairs))]
    matches = [p["matches"] for p in pairs]

    def one(e):
        s = max(0, e - window + 1)
        if e - s + 1 < 3:
            return e, None
        return e, ba_ref.ba_window(kps[s:e + 1], matches[s:e], stereo[s:e], rel[s:e], K, baseline, iters=iters)

    with ThreadPoolExecutor(max_workers=threads()) as ex:
        return dict(ex.map(one, ends))
