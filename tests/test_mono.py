"""Mono path (mono_slam.py:111-118 findEssentialMat + recoverPose).

CPU: the oracle against its golden vectors and against geometry (known-answer two-view
sets: the 5-point solver contains the true essential matrix, RANSAC + recoverPose return
the true pose on noise-free data).  GPU: the HIP kernels against the oracle — identical
status, RANSAC iteration-independent outputs (inlier mask, cheirality count) and E, R, t
within 1e-9 (both sides follow the same operation order in fp64; the tolerance allows for
libm vs device sqrt/log ulps)."""
import os

import numpy as np
import pytest
import torch

import mono_cases as mc
from conftest import GOLDEN, gpu_available


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "golden_mono.npz"))


def _skew(t):
    return np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])


# ------------------------------------------------------------------ oracle (CPU)
def test_golden_mono_reproduces(oracle_mod, golden):
    g = golden
    for i, (seed, n, noise, outl) in enumerate(mc.CASES):
        p0, p1, _, _ = mc.two_view(seed, n, noise, outl)
        st, E, mask, ni, _ = oracle_mod.find_essential(p0, p1, mc.F, (mc.CX, mc.CY))
        assert st == int(g[f"c{i}_status"]) and ni == int(g[f"c{i}_iters"])
        assert np.array_equal(mask, g[f"c{i}_mask"])
        assert np.array_equal(E, g[f"c{i}_E"])
        if st == 1:
            gd, R, t = oracle_mod.recover_pose(E, p0, p1, mc.F, (mc.CX, mc.CY))
            assert gd == int(g[f"c{i}_good"])
            assert np.array_equal(R, g[f"c{i}_R"]) and np.array_equal(t, g[f"c{i}_t"])
    K = g["K"]
    m = g["matches"]
    mk0 = g["kp0"][:, :2].astype(np.float32)[m[:, 0]]
    mk1 = g["kp1"][:, :2].astype(np.float32)[m[:, 1]]
    st, E, mask, ni, _ = oracle_mod.find_essential(mk0, mk1, K[0, 0], (K[0, 2], K[1, 2]))
    assert st == int(g["seq_status"]) and ni == int(g["seq_iters"]) and np.array_equal(E, g["seq_E"])


def test_five_point_contains_true_essential(oracle_mod):
    rng = np.random.default_rng(0)
    for trial in range(20):
        R = mc.rot(rng.normal(size=3) * 0.2)
        t = rng.normal(size=3)
        t /= np.linalg.norm(t)
        X = np.c_[rng.uniform(-2, 2, 5), rng.uniform(-2, 2, 5), rng.uniform(3, 10, 5)]
        X2 = X @ R.T + t
        x1, x2 = X[:, :2] / X[:, 2:], X2[:, :2] / X2[:, 2:]
        Ms = oracle_mod.five_point(x1, x2)
        Et = _skew(t) @ R
        Et /= np.linalg.norm(Et)
        assert 1 <= len(Ms) <= 10
        err = min(min(np.abs(M - Et).max(), np.abs(M + Et).max()) for M in Ms)
        assert err < 1e-8, (trial, err)
        for M in Ms:  # every solution: epipolar on the 5 points, rank 2, trace constraint
            h1, h2 = np.c_[x1, np.ones(5)], np.c_[x2, np.ones(5)]
            assert np.abs(np.einsum("ij,jk,ik->i", h2, M, h1)).max() < 1e-9
            assert abs(np.linalg.det(M)) < 1e-9
            assert np.abs(2 * M @ M.T @ M - np.trace(M @ M.T) * M).max() < 1e-9


@pytest.mark.parametrize("seed", [21, 22, 23, 24])
def test_ransac_recovers_true_pose(oracle_mod, seed):
    p0, p1, R, t = mc.two_view(seed, 400, noise=0.0, outliers=0.3)
    st, E, mask, ni, bg = oracle_mod.find_essential(p0, p1, mc.F, (mc.CX, mc.CY))
    assert st == 1 and bg >= 280
    g, Rr, tr = oracle_mod.recover_pose(E, p0, p1, mc.F, (mc.CX, mc.CY))
    assert np.abs(Rr - R).max() < 1e-4 and np.abs(tr - t).max() < 1e-3
    assert abs(np.linalg.det(Rr) - 1) < 1e-12 and abs(np.linalg.norm(tr) - 1) < 1e-12


def test_edge_sizes(oracle_mod):
    p0, p1, _, _ = mc.two_view(3, 4, 0, 0)
    assert oracle_mod.find_essential(p0, p1, mc.F, (mc.CX, mc.CY))[0] == -1
    st, E, mask, _, _ = oracle_mod.find_essential(p0[:0], p1[:0], mc.F, (mc.CX, mc.CY))
    assert st == -1
    p0, p1, R, t = mc.two_view(3, 5, 0, 0)
    st, E, mask, _, _ = oracle_mod.find_essential(p0, p1, mc.F, (mc.CX, mc.CY))
    assert st in (1, -2, 0)
    if st == 1:
        assert mask.all()


# ------------------------------------------------------------------ GPU parity


def _pack(sets, cap):
    B = len(sets)
    P0 = np.zeros((B, cap, 2), np.float32)
    P1 = np.zeros((B, cap, 2), np.float32)
    n = np.zeros(B, np.int32)
    for b, (p0, p1) in enumerate(sets):
        P0[b, :len(p0)] = p0
        P1[b, :len(p1)] = p1
        n[b] = len(p0)
    return torch.from_numpy(P0).cuda(), torch.from_numpy(P1).cuda(), torch.from_numpy(n).cuda()


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_gpu_essential_recover_matches_oracle(oracle_mod):
    from forest_slam_amd import _lib
    cap = 2048
    sets = [mc.two_view(*c)[:2] for c in mc.CASES] + [mc.two_view(40 + s, 300, 0.3, 0.2)[:2] for s in range(5)]
    ctx = _lib.Context(320, 200, max_batch=len(sets), stages=_lib.STAGE_MONO, kp_capacity=cap)
    P0, P1, n = _pack(sets, cap)
    E, mask, st = ctx.find_essential(P0, P1, n, mc.F, (mc.CX, mc.CY))
    R, t, T, g = ctx.recover_pose(E, P0, P1, n, mc.F, (mc.CX, mc.CY), e_status=st)
    torch.cuda.synchronize()
    E, mask, st = E.cpu().numpy(), mask.cpu().numpy(), st.cpu().numpy()
    R, t, T, g = R.cpu().numpy(), t.cpu().numpy(), T.cpu().numpy(), g.cpu().numpy()
    for b, (p0, p1) in enumerate(sets):
        k = len(p0)
        rst, rE, rmask, _, _ = oracle_mod.find_essential(p0, p1, mc.F, (mc.CX, mc.CY))
        assert st[b] == rst, (b, st[b], rst)
        if rst != 1:
            assert g[b] == -1 and np.array_equal(T[b], np.eye(4))
            continue
        assert np.abs(E[b] - rE).max() < 1e-9, b
        assert np.array_equal(mask[b, :k], rmask) and not mask[b, k:].any(), b
        rg, rR, rt = oracle_mod.recover_pose(rE, p0, p1, mc.F, (mc.CX, mc.CY))
        assert g[b] == rg, (b, g[b], rg)
        assert np.abs(R[b] - rR).max() < 1e-9 and np.abs(t[b] - rt).max() < 1e-9, b
        assert np.array_equal(T[b, :3, :3], R[b]) and np.array_equal(T[b, :3, 3], t[b])


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_gpu_mono_frontend_matches_golden(golden):
    """ORB -> BF -> gather -> findEssentialMat -> recoverPose through MonoFrontEnd on the
    golden frame pair (the oracle's outputs committed in golden_mono.npz)."""
    from forest_slam_amd import vo
    g = golden
    K = g["K"]
    fe = vo.MonoFrontEnd(320, 200, K, batch=1, nfeatures=300, device="cuda:0")
    fe.prime(torch.from_numpy(g["I0"]).cuda())
    T, st = fe.step(torch.from_numpy(g["I1"][None]).cuda())
    torch.cuda.synchronize()
    nm = int(fe.nmatch[0].item())
    assert np.array_equal(fe.matches[0, :nm].cpu().numpy(), g["matches"])
    assert int(st[0].item()) == int(g["seq_status"])
    assert np.abs(fe.E[0].cpu().numpy() - g["seq_E"]).max() < 1e-9
    assert np.array_equal(fe.mask[0, :nm].cpu().numpy(), g["seq_mask"])
    assert int(fe.ngood[0].item()) == int(g["seq_good"])
    assert np.abs(fe.R[0].cpu().numpy() - g["seq_R"]).max() < 1e-9
    assert np.abs(fe.t[0].cpu().numpy() - g["seq_t"]).max() < 1e-9


def _oracle_pool(fn, items):
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:  # ctypes calls drop the GIL
        return list(ex.map(fn, items))


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_gpu_mono_frontend_benchmark_shape_matches_oracle(oracle_mod):
    """VERDICT r2 missing #2: vo.MonoFrontEnd at the launch shape tools/bench_mono.py measures
    (configs[2]: 960x600, nfeatures 1000, B = 64) over 64 consecutive synthetic frame pairs,
    each pair against the oracle (ORB -> BF -> gather, mono_slam.py:106-108; findEssentialMat,
    :111; recoverPose, :112).  Two frames are blanked (no FAST corners), so three pairs of the
    batch have no matches and take the -1 status.  Identical matches, statuses and inlier
    masks; E, R, t within 1e-9.  Then the -1 / -2 edge sets (4 and 5 points) inside one
    B = 64 fvo_find_essential launch of the same context."""
    from forest_slam_amd import synth, vo
    B, W, H, NF = 64, 960, 600, 1000
    seq = synth.StereoSequence(seed=7, n_frames=B + 1, W=W, H=H, device="cuda", start=30)
    I, _ = seq.frames(range(B + 1))
    I = I.clone()
    I[20] = 128
    I[21] = 128
    torch.cuda.synchronize()
    K = seq.K
    f, pp = float(K[0, 0]), (float(K[0, 2]), float(K[1, 2]))
    fe = vo.MonoFrontEnd(W, H, K, batch=B, nfeatures=NF, device="cuda:0")
    fe.prime(I[0])
    T, st = fe.step(I[1:])
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    E, mask, R, t = (x.cpu().numpy() for x in (fe.E, fe.mask, fe.R, fe.t))
    M, nm, good = fe.matches.cpu().numpy(), fe.nmatch.cpu().numpy(), fe.ngood.cpu().numpy()
    imgs = I.cpu().numpy()
    feats = _oracle_pool(lambda im: oracle_mod.orb_detect_compute(im, NF), list(imgs))

    def pair(b):
        (k0, d0), (k1, d1) = feats[b], feats[b + 1]
        m = oracle_mod.bf_match(d0, d1) if len(d0) and len(d1) else np.zeros((0, 3), np.int32)
        mk0 = k0[:, :2].astype(np.float32)[m[:, 0]] if len(m) else np.zeros((0, 2), np.float32)
        mk1 = k1[:, :2].astype(np.float32)[m[:, 1]] if len(m) else np.zeros((0, 2), np.float32)
        rst, rE, rmask, _, _ = oracle_mod.find_essential(mk0, mk1, f, pp)
        rp = oracle_mod.recover_pose(rE, mk0, mk1, f, pp) if rst == 1 else None
        return m, rst, rE, rmask, rp

    ref = _oracle_pool(pair, range(B))
    sts = [r[1] for r in ref]
    assert sts.count(-1) >= 3 and sts.count(1) >= 50, sts
    for b, (m, rst, rE, rmask, rp) in enumerate(ref):
        k = len(m)
        assert nm[b] == k and np.array_equal(M[b, :k], m), b
        assert st[b] == rst, (b, st[b], rst)
        if rst != 1:
            assert good[b] == -1 and np.array_equal(T[b].cpu().numpy(), np.eye(4)), b
            continue
        assert np.abs(E[b] - rE).max() < 1e-9, b
        assert np.array_equal(mask[b, :k], rmask) and not mask[b, k:].any(), b
        rg, rR, rt = rp
        assert good[b] == rg, (b, good[b], rg)
        assert np.abs(R[b] - rR).max() < 1e-9 and np.abs(t[b] - rt).max() < 1e-9, b

    # -1 (no points, 4 points) and -2 (5 points, several solutions) beside ordinary sets
    fives = [s for s in range(3, 400) if oracle_mod.find_essential(*mc.two_view(s, 5, 0.0, 0.0)[:2], mc.F,
                                                                   (mc.CX, mc.CY))[0] == -2][:4]
    sets = [mc.two_view(1, 0)[:2], mc.two_view(2, 4)[:2]] + [mc.two_view(s, 5, 0.0, 0.0)[:2] for s in fives]
    sets += [mc.two_view(60 + s, 300 + 7 * s, 0.4, 0.3)[:2] for s in range(B - len(sets))]
    P0, P1, n = _pack(sets, fe.cap)
    E2, mask2, st2 = fe.ctx.find_essential(P0, P1, n, mc.F, (mc.CX, mc.CY))
    torch.cuda.synchronize()
    E2, mask2, st2 = E2.cpu().numpy(), mask2.cpu().numpy(), st2.cpu().numpy()
    want = _oracle_pool(lambda pq: oracle_mod.find_essential(pq[0], pq[1], mc.F, (mc.CX, mc.CY)), sets)
    assert [w[0] for w in want[:6]] == [-1, -1, -2, -2, -2, -2]
    for b, (rst, rE, rmask, _, _) in enumerate(want):
        assert st2[b] == rst, (b, st2[b], rst)
        if rst == 1:
            assert np.abs(E2[b] - rE).max() < 1e-9, b
            assert np.array_equal(mask2[b, :len(sets[b][0])], rmask), b


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_gpu_mono_overlapped_steps_equal_in_order():
    """MonoFrontEnd(overlap=True) -- ORB + BF of step k+1 on a side stream beside step k's
    essential-matrix stage, double-buffered -- returns exactly the in-order results over
    several steps (incl. a short last step)."""
    from forest_slam_amd import synth, vo
    B, W, H = 8, 640, 400
    seq = synth.StereoSequence(seed=5, n_frames=3 * B + 1, W=W, H=H, device="cuda", start=40)
    I, _ = seq.frames(range(3 * B + 1))
    torch.cuda.synchronize()
    outs = []
    for ov in (False, True):
        fe = vo.MonoFrontEnd(W, H, seq.K, batch=B, nfeatures=500, device="cuda:0", overlap=ov)
        fe.prime(I[0])
        Ts, sts = [], []
        for s, e in ((1, 1 + B), (1 + B, 1 + 2 * B), (1 + 2 * B, 3 * B + 1 - 3)):
            T, st = fe.step(I[s:e].contiguous())
            Ts.append(T.clone())
            sts.append(st.clone())
        torch.cuda.synchronize()
        outs.append((torch.cat(Ts).cpu().numpy(), torch.cat(sts).cpu().numpy()))
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][0], outs[1][0])
