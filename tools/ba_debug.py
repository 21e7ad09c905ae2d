"""Debug helper: GPU BA vs oracle on the test problems, max deviations (dev tool)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np, torch
import ba_synth, ba_ref
from forest_slam_amd import _lib
for (n, seed, drop, K) in [(10, 0, 0.0, 10), (12, 3, 0.05, 10), (20, 5, 0.0, 20)]:
    p = ba_synth.clean_problem(n=n, seed=seed, drop=drop, n_pts=2500)
    F, cap = p["kp"].shape[:2]
    nw = n - 2
    ctx = _lib.Context(64, 64, max_batch=nw, stages=_lib.STAGE_BA, kp_capacity=cap, ba_window=K)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    args = [t(p[k]) for k in ("kp", "nkp", "matches", "nmatch", "stereo", "T_rel")]
    Tout, stats = ctx.ba_windows(*args, 2, nw, 0, p["K"], p["B"], iterations=10)
    Tout, stats = Tout.cpu().numpy(), stats.cpu().numpy()
    dT, dc = 0, 0
    for w in range(nw):
        e = 2 + w; s = max(0, e - K + 1)
        kps, m, st, rel = ba_synth.oracle_lists(p, s, e)
        r = ba_ref.ba_window(kps, m, st, rel, p["K"], p["B"], iters=10)
        dT = max(dT, np.abs(Tout[w] - r["rel"][-1]).max()); dc = max(dc, abs(stats[w][1] - r["cost"]) / r["cost0"])
    print(n, seed, drop, K, "max dT", dT, "max dcost/cost0", dc)
