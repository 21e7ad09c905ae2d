"""Dev tool: run the GPU front end on a synthetic sequence and dump per-frame BA inputs
(keypoints, matches, stereo points, PnP transforms, statuses, BA outputs) for offline analysis."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import numpy as np, torch
from forest_slam_amd import synth, vo
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda", 0)
seq = synth.StereoSequence(seed=100, n_frames=n, W=960, H=600, device=dev)
L, R = seq.frames(range(n))
fe = vo.StereoFrontEnd(960, 600, seq.K, synth.DIST_L, synth.BASELINE, batch=32, nfeatures=1000, device=dev, ba_window=10)
fe.prime(L[0], R[0])
kp = [fe.hkp[fe.ba_window - 2].cpu().numpy()[:, :6].copy()]
nkp = [int(fe.hnkp[fe.ba_window - 2])]
M, NM, ST, T, S, TB, BS = [], [], [], [], [], [], []
for s in range(1, n, 32):
    e = min(s + 32, n)
    Tb, st = fe.step(L[s:e], R[s:e])
    k = e - s
    a, b = fe.ba_window - 2, fe.ba_window - 1
    # history has already slid; recompute what we need from the step buffers
    kp += [x[:, :6].copy() for x in fe.kp[:k].cpu().numpy()]
    nkp += list(fe.cnt[:k].cpu().numpy())
    M += list(fe.matches[:k].cpu().numpy()); NM += list(fe.nmatch[:k].cpu().numpy())
    T += list(fe.T[:k].cpu().numpy()); S += list(st.cpu().numpy())
    TB += list(Tb.cpu().numpy()); BS += list(fe.ba_stats[:k].cpu().numpy())
    ST += list(fe.ctx.keypoint_stereo(fe.disp[:k], fe.q_kp[:k], fe.cnt[:k] * 0 + torch.tensor([int(x) for x in nkp[-k - 1:-1]], dtype=torch.int32, device=dev), seq.K, synth.BASELINE).cpu().numpy())
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "seqdump.npz"), kp=np.array(kp, np.float32), nkp=np.array(nkp),
                    matches=np.array(M), nmatch=np.array(NM), stereo=np.array(ST), T=np.array(T), status=np.array(S),
                    Tba=np.array(TB), ba_stats=np.array(BS), t=seq.t, T_wc=seq.T_wc, K=seq.K)
print("dumped", n)
