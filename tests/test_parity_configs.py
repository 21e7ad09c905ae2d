"""End-to-end GPU parity at BASELINE.json's configurations (VERDICT r1 "untested configs").

* configs[3] per-GPU workload: 960x600, ORB nfeatures=1000, local BA K = 10, StereoFrontEnd
  batches of 4 (windows span step boundaries);
* configs[4]: synthetic 1920x1080 forest, nfeatures=2000, local BA K = 20.

Checker: the oracle pipeline (tests/pipeline_ref.py: oracle.frame_pose per frame pair =
stereo_slam.py:232-303, then ba_ref.ba_window per window).  Bit-exact: BF match rows,
SGBM disparities, float32 3D points; PnP relative transforms within 1e-4 (north_star);
local-BA transforms within 1e-8 of the float64 specification (initialised, like the
product, with the product's PnP transforms: a RANSAC model can flip between two
implementations on an ill-conditioned EPnP subset).  Frames are rendered on
the GPU and copied to the host, so both sides see identical bytes.
"""
import numpy as np
import pytest
import torch

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]


def _run(oracle_mod, W, H, nfeatures, Kw, n, batch, seed, start, ba_ends):
    import ba_ref
    import pipeline_ref
    from forest_slam_amd import synth, vo
    seq = synth.StereoSequence(seed=seed, n_frames=n, W=W, H=H, device="cuda", start=start)
    Ls, Rs = seq.frames(range(n))
    torch.cuda.synchronize()
    fr = [(Ls[i].cpu().numpy(), Rs[i].cpu().numpy()) for i in range(n)]
    fe = vo.StereoFrontEnd(W, H, seq.K, synth.DIST_L, synth.BASELINE, batch=batch, nfeatures=nfeatures,
                           ba_window=Kw)
    fe.prime(Ls[0], Rs[0])
    got = dict(T_ba=[], T_pnp=[], st=[], m=[], disp=[], P3=[])
    for s in range(1, n, batch):
        e = min(s + batch, n)
        k = e - s
        T, st = fe.step(Ls[s:e], Rs[s:e])
        torch.cuda.synchronize()
        got["T_ba"].append(T.cpu().numpy().copy())
        got["T_pnp"].append(fe.T[:k].cpu().numpy().copy())
        got["st"].append(st.cpu().numpy().copy())
        for i in range(k):
            got["m"].append(fe.matches[i, :int(fe.nmatch[i].item())].cpu().numpy().copy())
            got["disp"].append(fe.disp[i].cpu().numpy().copy())
            got["P3"].append(fe.P3[i, :int(fe.npts[i].item())].cpu().numpy().copy())
    T_ba, T_pnp, st = (np.concatenate(got[k]) for k in ("T_ba", "T_pnp", "st"))
    del fe
    pairs, kps = pipeline_ref.sequence(oracle_mod, fr, seq.K, synth.DIST_L, synth.BASELINE, nfeatures)
    for j, ref in enumerate(pairs):
        assert np.array_equal(got["m"][j], ref["matches"]), f"pair {j}: BF matches differ"
        bad = np.argwhere(got["disp"][j] != ref["disp16"])
        assert len(bad) == 0, f"pair {j}: {len(bad)} disparity px differ, first {bad[:4]}"
        assert np.array_equal(got["P3"][j], ref["P3"]), f"pair {j}: 3D points differ"
        if ref["T"] is None:
            assert st[j] == -1
            continue
        assert st[j] == int(ref["ok"])
        assert np.abs(T_pnp[j] - ref["T"]).max() <= 1e-4 * max(1.0, np.abs(ref["T"]).max()), f"pair {j}: PnP pose"
    refs = pipeline_ref.ba_windows(ba_ref, pairs, kps, T_pnp, seq.K, synth.BASELINE, Kw, ba_ends)
    for e, ref in refs.items():
        if ref is None:
            assert np.array_equal(T_ba[e - 1], T_pnp[e - 1])
        else:
            assert np.abs(T_ba[e - 1] - ref["rel"][-1]).max() < 1e-8, f"BA window ending at frame {e}"
    return pairs


def test_config3_600p_1000kp_local_ba_k10(oracle_mod):
    """configs[3]'s per-GPU workload: 14 frames, batch 4, every window K = 10 checked."""
    n = 14
    pairs = _run(oracle_mod, 960, 600, 1000, 10, n, 4, seed=12, start=200, ba_ends=list(range(1, n)))
    assert min(len(p["matches"]) for p in pairs) > 100


def test_config5_1080p_2000kp_local_ba_k20(oracle_mod):
    """configs[4]: 1920x1080, 2000 keypoints per frame, K = 20 (the full windows ending at
    frames 19 and 20 plus two short ones), batch 8."""
    n = 21
    pairs = _run(oracle_mod, 1920, 1080, 2000, 20, n, 8, seed=13, start=300, ba_ends=[1, 2, 19, 20])
    assert min(len(p["kp0"]) for p in pairs) > 1500
