"""Reads the stage stamps of a tools/refine_probe_patch.py build (FVO_LIB) after three steps
of the bench's front end: mean / max per stage over the batch, in us (100 MHz clock)."""
import os, sys, json, torch, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from forest_slam_amd import synth, vo
hd = "--hd" in sys.argv
W, H, NF, K, B = (1920, 1080, 2000, 20, 32) if hd else (960, 600, 1000, 10, 64)
caps = dict(ba_max_landmarks=8192, ba_max_obs=65536) if hd else {}
seq = synth.StereoSequence(seed=0, n_frames=B + 1, W=W, H=H, device="cuda")
L, R = seq.frames(range(B + 1))
fe = vo.StereoFrontEnd(W, H, seq.K, synth.DIST_L, synth.BASELINE, batch=B, nfeatures=NF, ba_window=K, **caps)
fe.prime(L[0], R[0])
for _ in range(3):
    fe.step(L[1:], R[1:])
torch.cuda.synchronize()
m = fe.ctx.debug_buffer(7).view(torch.float64).view(B, -1, 6).numpy()
mi = m.shape[1]
t = m[:, mi - 2:, :].reshape(B, 12)[:, :9]
d = np.diff(t[:, [0, 1, 2, 3, 4, 5]], axis=1) * 10 / 1e3  # us (100 MHz)
print("stages us (compact, accum, dlt, init, LM): mean", d.mean(0).round(1), "max", d.max(0).round(1))
print("iters mean", t[:, 6].mean(), "max", t[:, 6].max(), "ninl mean", t[:, 8].mean())
