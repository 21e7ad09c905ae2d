"""Minimal SGBM launch on cuda:0 (960x600, 2 pairs) checked against the oracle; for diagnosing launch failures."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np, torch
import oracle
from forest_slam_amd import _lib, synth
seq = synth.StereoSequence(seed=0, n_frames=2, W=960, H=600, device="cpu")
fr = [tuple(x.numpy() for x in seq.frame(i)) for i in range(2)]
L = np.stack([f[0] for f in fr]); R = np.stack([f[1] for f in fr])
ctx = _lib.Context(960, 600, max_batch=2, stages=_lib.STAGE_SGBM)
print("ctx ok", flush=True)
d = ctx.sgbm(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda())
print("launched", flush=True)
torch.cuda.synchronize()
d = d.cpu().numpy()
for i in range(2):
    print(i, int((d[i] != oracle.sgbm(L[i], R[i])).sum()), "px differ", flush=True)
