"""BA stage time alone per LPC variant: the bench's front end (960x600, 1000 features, K=10),
per-kernel-group times (HIP events) over 3 steps.  Prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from forest_slam_amd import synth, vo  # noqa: E402

B = 64
seq = synth.StereoSequence(seed=0, n_frames=B + 1, W=960, H=600, device="cuda")
L, R = seq.frames(range(B + 1))
fe = vo.StereoFrontEnd(960, 600, seq.K, synth.DIST_L, synth.BASELINE, batch=B, nfeatures=1000, ba_window=10)
fe.prime(L[0], R[0])
for _ in range(2):
    fe.step(L[1:], R[1:])
torch.cuda.synchronize()
fe.ctx.timing_enable(None)
for _ in range(3):
    fe.step(L[1:], R[1:])
torch.cuda.synchronize()
st = fe.ctx.timing_read()
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("FVO_")},
                  "ms": {k: round(v[0] / 3, 3) for k, v in st.items() if k.startswith(("ba", "pnp"))}}), flush=True)
