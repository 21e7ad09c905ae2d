"""Per-frame PnP RANSAC state (best inlier count, iteration bound) after the bench's steady-state
step, 600p batch 64 (tooling: how much of the 1000-iteration budget round 2 really runs)."""
import os, sys, json, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from forest_slam_amd import synth, vo
B = 64
seq = synth.StereoSequence(seed=0, n_frames=B + 1, W=960, H=600, device="cuda")
L, R = seq.frames(range(B + 1))
fe = vo.StereoFrontEnd(960, 600, seq.K, synth.DIST_L, synth.BASELINE, batch=B, nfeatures=1000, ba_window=10)
fe.prime(L[0], R[0])
for step in range(3):
    fe.step(L[1:], R[1:])
    torch.cuda.synchronize()
    st = fe.ctx.debug_buffer(8).view(torch.int32).view(-1, 4)[:B]
    print(json.dumps({"step": step, "niters": st[:, 1].tolist(), "maxGood": st[:, 0].tolist(), "n": st[:, 3].tolist()}))
