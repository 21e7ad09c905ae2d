"""Generate tests/golden/golden_mono.npz with the oracle: findEssentialMat + recoverPose
(mono_slam.py:111-112) on seeded two-view sets (tests/mono_cases.py) and on ORB+BF
matches of two synthetic forest frames.  No reference fixture exists for this path
(the reference has no tests; OpenCV is absent), so these pin the oracle against
regressions.  Regenerate only on a deliberate oracle change:
    python tests/golden/make_golden_mono.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import oracle  # noqa: E402
import mono_cases as mc  # noqa: E402
from forest_slam_amd import synth  # noqa: E402


def main():
    oracle.build()
    out = {}
    for i, (seed, n, noise, outl) in enumerate(mc.CASES):
        p0, p1, _, _ = mc.two_view(seed, n, noise, outl)
        st, E, mask, ni, bg = oracle.find_essential(p0, p1, mc.F, (mc.CX, mc.CY))
        g, R, t = oracle.recover_pose(E, p0, p1, mc.F, (mc.CX, mc.CY)) if st == 1 else (-1, np.eye(3), np.zeros(3))
        out.update({f"c{i}_status": np.int32(st), f"c{i}_E": E, f"c{i}_mask": mask, f"c{i}_iters": np.int32(ni),
                    f"c{i}_good": np.int32(g), f"c{i}_R": R, f"c{i}_t": t})
    W, H = 320, 200
    seq = synth.StereoSequence(seed=5, n_frames=4, W=W, H=H, device="cpu", start=100)
    I0 = seq.frame(0)[0].numpy()
    I1 = seq.frame(3)[0].numpy()
    kp0, d0 = oracle.orb_detect_compute(I0, 300)
    kp1, d1 = oracle.orb_detect_compute(I1, 300)
    m = oracle.bf_match(d0, d1)
    mk0 = kp0[:, :2].astype(np.float32)[m[:, 0]]
    mk1 = kp1[:, :2].astype(np.float32)[m[:, 1]]
    K = seq.K
    st, E, mask, ni, bg = oracle.find_essential(mk0, mk1, K[0, 0], (K[0, 2], K[1, 2]))
    g, R, t = oracle.recover_pose(E, mk0, mk1, K[0, 0], (K[0, 2], K[1, 2]))
    out.update(I0=I0, I1=I1, K=K, kp0=kp0, kp1=kp1, matches=m, seq_status=np.int32(st), seq_E=E, seq_mask=mask,
               seq_iters=np.int32(ni), seq_good=np.int32(g), seq_R=R, seq_t=t)
    np.savez_compressed(os.path.join(HERE, "golden_mono.npz"), **out)
    print("golden_mono.npz:", len(m), "matches, status", st, "iters", ni, "inliers", bg, "cheiral", g)


if __name__ == "__main__":
    main()
