"""Generate the committed golden vectors (tests/golden/golden_small.npz) with the oracle.

The reference has no tests or fixtures for this path and OpenCV is not installed here, so
these vectors come from the oracle (the C++ restatement of the reference's OpenCV calls)
on seeded synthetic inputs; they pin the oracle against regressions and are the fixed
expected outputs the GPU parity tests also check.  Regenerate only on a deliberate oracle
change:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import oracle  # noqa: E402
from forest_slam_amd import synth  # noqa: E402


def main():
    oracle.build()
    W, H = 320, 200
    seq = synth.StereoSequence(seed=11, n_frames=3, W=W, H=H, device="cpu")
    (L0, R0), (L1, R1) = [tuple(x.numpy() for x in seq.frame(i)) for i in range(2)]
    kp0, d0 = oracle.orb_detect_compute(L0, 300)
    kp1, d1 = oracle.orb_detect_compute(L1, 300)
    m = oracle.bf_match(d0, d1)
    disp = oracle.sgbm(L0, R0, num_disp=64)
    mk0 = kp0[:, :2].astype(np.float32)[m[:, 0]]
    mk1 = kp1[:, :2].astype(np.float32)[m[:, 1]]
    P3, p2, _ = oracle.backproject(oracle.disparity_map(disp), mk0, mk1, seq.K, synth.BASELINE)
    ok, rv, tv, inl, ni, bg = oracle.solve_pnp_ransac(P3, p2, seq.K, synth.DIST_L)
    np.savez_compressed(os.path.join(HERE, "golden_small.npz"), L0=L0, R0=R0, L1=L1, R1=R1, K=seq.K, kp0=kp0, d0=d0,
                        kp1=kp1, d1=d1, matches=m, disp16=disp, P3=P3, p2=p2, pnp_ok=np.int32(ok), rvec=rv, tvec=tv,
                        inliers=inl, ransac_iters=np.int32(ni))
    print("golden_small.npz:", len(kp0), len(kp1), len(m), len(P3), ok, ni, bg)


if __name__ == "__main__":
    main()
