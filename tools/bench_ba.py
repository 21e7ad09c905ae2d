"""BA stage time alone (tooling): the bench's front end at a configuration, the BA kernel
group's time (HIP events) over 3 steps; the library build is FVO_LIB's (tools/build_variant.py)
or the in-tree one.  Prints one JSON line.
    python tools/bench_ba.py [--hd]    (--hd: 1920x1080, 2000 features, K=20, 32 frames)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from forest_slam_amd import synth, vo  # noqa: E402

hd = "--hd" in sys.argv
W, H, NF, K, B = (1920, 1080, 2000, 20, 32) if hd else (960, 600, 1000, 10, 64)
caps = dict(ba_max_landmarks=8192, ba_max_obs=65536) if hd else {}
seq = synth.StereoSequence(seed=0, n_frames=B + 1, W=W, H=H, device="cuda")
L, R = seq.frames(range(B + 1))
fe = vo.StereoFrontEnd(W, H, seq.K, synth.DIST_L, synth.BASELINE, batch=B, nfeatures=NF, ba_window=K, **caps)
fe.prime(L[0], R[0])
for _ in range(2):
    T, _ = fe.step(L[1:], R[1:])
torch.cuda.synchronize()
fe.ctx.timing_enable(None)
for _ in range(3):
    T, _ = fe.step(L[1:], R[1:])
torch.cuda.synchronize()
st = fe.ctx.timing_read()
print(json.dumps({"lib": os.environ.get("FVO_LIB", "in-tree"), "config": f"{W}x{H} K={K} B={B}",
                  "T_checksum": float(T.double().abs().sum().item()),
                  "ms": {k: round(v[0] / 3, 3) for k, v in st.items() if k.startswith(("ba", "pnp"))}}), flush=True)
