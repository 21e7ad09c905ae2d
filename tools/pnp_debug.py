"""Debug helper: GPU vs oracle PnP on the frames of test_gpu_frontend_local_ba (dev tool)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np, torch
import oracle
from forest_slam_amd import synth, vo
W, H, n = 640, 400, 6
seq = synth.StereoSequence(seed=9, n_frames=n, W=W, H=H, device="cpu", start=150)
fr = [tuple(x.numpy() for x in seq.frame(i)) for i in range(n)]
fe = vo.StereoFrontEnd(W, H, seq.K, synth.DIST_L, synth.BASELINE, batch=2, nfeatures=500, ba_window=4)
Ls = torch.from_numpy(np.stack([f[0] for f in fr])).cuda()
Rs = torch.from_numpy(np.stack([f[1] for f in fr])).cuda()
fe.prime(Ls[0], Rs[0])
for s in range(1, n, 2):
    fe.step(Ls[s:s + 2], Rs[s:s + 2])
    for i in range(2):
        j = s - 1 + i
        r = oracle.frame_pose(fr[j][0], fr[j][1], fr[j + 1][0], seq.K, synth.DIST_L, synth.BASELINE, 500)
        npt = int(fe.npts[i].item())
        P3 = fe.P3[i, :npt].cpu().numpy(); p2 = fe.p2[i, :npt].cpu().numpy()
        print("pair", j, "npts", npt, len(r["P3"]), "P3 eq", np.array_equal(P3, r["P3"]), "p2 eq", np.array_equal(p2, r["p2"]))
        ok, rv, tv, inl, iters, bg = oracle.solve_pnp_ransac(r["P3"], r["p2"], seq.K, synth.DIST_L)
        ginl = np.nonzero(fe.inl[i, :npt].cpu().numpy())[0]
        print("   oracle ok", ok, "iters", iters, "best", bg, "ninl", len(inl), "| gpu st", int(fe.status[i]), "ninl", len(ginl),
              "same inl", np.array_equal(np.sort(inl), ginl))
        print("   rv", rv, fe.rvec[i].cpu().numpy(), "\n   tv", tv, fe.tvec[i].cpu().numpy())
