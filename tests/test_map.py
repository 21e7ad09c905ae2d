"""Map accumulation: the per-frame map update of stereo_slam.py:308-318
(cum @ [P; 1], PointCloud2 FLOAT32 packing) and mono_slam.py:144-164 / gt_mapping.py:62-66
(Open3D voxel_down_sample(0.5)).  Open3D is not installed here: the oracle (oracle/map_ref.cpp)
restates VoxelDownSample and is checked against an independent NumPy/dict restatement of the
same algorithm ("parity unpinned" against Open3D itself; its output order, an unordered_map's,
is unspecified, so voxels are compared in index order).  CPU: oracle vs NumPy.  GPU: the HIP
kernels bit-exact against the oracle."""
import numpy as np
import pytest
import torch

from conftest import gpu_available


def _cloud(n, seed, spread=20.0):
    rng = np.random.default_rng(seed)
    P = rng.standard_normal((n, 3)) * spread
    P[: n // 4] = np.round(P[: n // 4] * 2) / 2  # points exactly on voxel boundaries
    return P.astype(np.float32)


def _pose(seed):
    rng = np.random.default_rng(seed)
    a, b = rng.uniform(-np.pi, np.pi, 2)
    Rz = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
    Rx = np.array([[1, 0, 0], [0, np.cos(b), -np.sin(b)], [0, np.sin(b), np.cos(b)]])
    T = np.eye(4)
    T[:3, :3] = Rz @ Rx
    T[:3, 3] = rng.uniform(-50, 50, 3)
    return T


def _voxel_numpy(P, v):
    """Open3D 0.17 VoxelDownSample restated with a dict (insertion-order sums)."""
    vmin = P.min(axis=0) - v * 0.5
    acc = {}
    for p in P:
        key = tuple(int(np.floor(c)) for c in (p - vmin) / v)
        s = acc.setdefault(key, [0.0, 0.0, 0.0, 0])
        s[0] += p[0]; s[1] += p[1]; s[2] += p[2]; s[3] += 1
    return np.array([[s[0] / s[3], s[1] / s[3], s[2] / s[3]] for _, s in sorted(acc.items())]).reshape(-1, 3)


def test_map_transform_oracle_matches_numpy(oracle_mod):
    P, T = _cloud(5000, 1), _pose(2)
    o64, o32 = oracle_mod.map_transform(P, T)
    ref = (T @ np.hstack((P, np.ones((len(P), 1)))).T)[:3].T  # stereo_slam.py:308-311
    assert np.allclose(o64, ref, rtol=0, atol=1e-12 * np.abs(ref).max())
    assert np.mean(o32 == ref.astype(np.float32)) > 0.999


@pytest.mark.parametrize("v", [0.5, 0.3])
def test_voxel_oracle_matches_numpy(oracle_mod, v):
    P = _cloud(3000, 3, spread=3.0).astype(np.float64)
    assert np.array_equal(oracle_mod.voxel_down_sample(P, v), _voxel_numpy(P, v))


def test_voxel_oracle_known_answers(oracle_mod):
    assert oracle_mod.voxel_down_sample(np.zeros((0, 3)), 0.5).shape == (0, 3)
    one = np.array([[1.25, -3.0, 7.5]])
    assert np.array_equal(oracle_mod.voxel_down_sample(one, 0.5), one)
    # min bound - v/2 puts the minimum point at the centre of voxel 0: these two share it
    two = np.array([[0.0, 0.0, 0.0], [0.2, 0.1, -0.1]])
    assert np.array_equal(oracle_mod.voxel_down_sample(two, 0.5), [[0.1, 0.05, -0.05]])


def _ctx():
    from forest_slam_amd import _lib
    return _lib.Context(64, 64, max_batch=1, stages=_lib.STAGE_BF, kp_capacity=64)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_gpu_map_transform_matches_oracle(oracle_mod):
    ctx = _ctx()
    B, cap = 5, 1200
    counts = [1000, 0, 1200, 37, 999]
    P = np.zeros((B, cap, 3), np.float32)
    for b in range(B):
        P[b] = _cloud(cap, 10 + b)
    T = np.stack([_pose(20 + b) for b in range(B)])
    M = sum(counts) + 100
    m64 = torch.zeros((M, 3), dtype=torch.float64, device="cuda")
    m32 = torch.zeros((M, 3), dtype=torch.float32, device="cuda")
    cnt = torch.tensor([100], dtype=torch.int32, device="cuda")  # append after 100 existing points
    ctx.map_transform(torch.from_numpy(P).cuda(), torch.tensor(counts, dtype=torch.int32, device="cuda"),
                      torch.from_numpy(T).cuda(), cnt, m64, m32)
    assert int(cnt.item()) == M
    g64, g32 = m64.cpu().numpy(), m32.cpu().numpy()
    assert not g64[:100].any()
    o = 100
    for b in range(B):
        w64, w32 = oracle_mod.map_transform(P[b, :counts[b]], T[b])
        assert np.array_equal(g64[o:o + counts[b]], w64) and np.array_equal(g32[o:o + counts[b]], w32), b
        o += counts[b]
    # overflow: points past map_cap are dropped, the count still advances
    small = torch.zeros((50, 3), dtype=torch.float32, device="cuda")
    cnt = torch.zeros((1,), dtype=torch.int32, device="cuda")
    ctx.map_transform(torch.from_numpy(P[:1]).cuda(), torch.tensor([1000], dtype=torch.int32, device="cuda"),
                      torch.from_numpy(T[:1]).cuda(), cnt, None, small)
    assert int(cnt.item()) == 1000
    assert np.array_equal(small.cpu().numpy(), oracle_mod.map_transform(P[0, :50], T[0])[1])


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_gpu_voxel_down_sample_matches_oracle(oracle_mod):
    ctx = _ctx()
    cases = [_cloud(200_000, 5).astype(np.float64), _cloud(3000, 6, spread=0.05).astype(np.float64),
             np.array([[1.0, 2.0, 3.0]]), np.repeat([[0.3, 0.3, 0.3]], 700, axis=0)]
    # a transformed lidar-like map (mono_slam.py:148-155)
    o64, _ = oracle_mod.map_transform(_cloud(50_000, 7, spread=30.0), _pose(8))
    cases.append(o64)
    for v in (0.5, 0.1):
        for P in cases:
            out, n, st = ctx.voxel_down_sample(torch.from_numpy(P).cuda(), v)
            want = oracle_mod.voxel_down_sample(P, v)
            assert int(st.item()) == 0
            assert int(n.item()) == len(want), (len(P), v)
            assert np.array_equal(out[:len(want)].cpu().numpy(), want), (len(P), v)
    out, n, st = ctx.voxel_down_sample(torch.zeros((0, 3), dtype=torch.float64, device="cuda"), 0.5)
    assert int(n.item()) == 0


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_gpu_point_map_mono_update_matches_oracle(oracle_mod):
    """mono_slam.py:144-164: cloud -> pose -> voxel_down_sample(0.5) -> appended to the map."""
    from forest_slam_amd.mapping import PointMap
    pm = PointMap(100_000)
    want = []
    for k in range(3):
        cloud, T = _cloud(20_000, 40 + k, spread=10.0), _pose(50 + k)
        pm.add_cloud(cloud, T, 0.5)
        o64, _ = oracle_mod.map_transform(cloud, T)
        want.append(oracle_mod.voxel_down_sample(o64, 0.5))
    want = np.concatenate(want)
    assert np.array_equal(pm.cloud64(), want)
    assert np.array_equal(pm.cloud32(), want.astype(np.float32))


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_gpu_point_map_overflow_is_reported():
    """an append past the capacity is surfaced (check=True raises at once,
    overflowed() / len() report it) instead of silently dropping later batches."""
    from forest_slam_amd.mapping import PointMap
    pm = PointMap(capacity=100, device="cuda:0")
    P = torch.from_numpy(_cloud(80, 3)).cuda().reshape(1, 80, 3)
    T = np.eye(4)[None]
    pm.add_frames(P, torch.tensor([80], dtype=torch.int32, device="cuda"), T, check=True)
    assert len(pm) == 80 and not pm.overflowed()
    with pytest.raises(RuntimeError, match="overflow"):
        pm.add_frames(P, torch.tensor([80], dtype=torch.int32, device="cuda"), T, check=True)
    assert pm.overflowed()


def _chain_ref(T, S, N, cum0):
    """stereo_slam.py:292-306 restated per sequence: cum = cum @ T for posed frames
    (status >= 0), summed over k ascending without contraction (fvo_chain_poses' order)."""
    cum = cum0.copy()
    out = np.zeros_like(T)
    nout = np.zeros_like(N)
    for s in range(T.shape[0]):
        c = cum[s]
        for f in range(T.shape[1]):
            if S[s, f] >= 0:
                t = T[s, f]
                c = np.array([[((c[i, 0] * t[0, j] + c[i, 1] * t[1, j]) + c[i, 2] * t[2, j]) + c[i, 3] * t[3, j]
                               for j in range(4)] for i in range(4)])
                nout[s, f] = N[s, f]
            out[s, f] = c
        cum[s] = c
    return out, nout, cum


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_chain_poses_matches_reference_chain():
    """fvo_chain_poses (the multi-sequence map's placing poses on the device): per sequence
    cum = cum @ T for every posed frame (status >= 0; -1 = the < 6 points skip, -2 padding, -3
    overflow leave it unchanged), carried across calls; equal to the ascending-k restatement bit
    for bit and to eval.chain's np.dot chain within 1e-12; points of unposed frames zeroed."""
    from forest_slam_amd import _lib
    from forest_slam_amd import eval as ev
    rng = np.random.default_rng(9)
    S_, n = 5, 7
    T = np.stack([[_pose(100 * s + f) for f in range(2 * n)] for s in range(S_)])
    T[..., :3, 3] *= 0.01
    St = rng.choice([1, 1, 1, 0, -1, -2, -3], size=(S_, 2 * n)).astype(np.int32)
    N = rng.integers(0, 900, size=(S_, 2 * n)).astype(np.int32)
    ctx = _lib.Context(64, 64, max_batch=1, stages=_lib.STAGE_BF, kp_capacity=64, device="cuda:0")
    cum = torch.eye(4, dtype=torch.float64, device="cuda:0").repeat(S_, 1, 1).contiguous()
    ref_cum = np.tile(np.eye(4), (S_, 1, 1))
    for h in range(2):  # two calls: the chain carries over
        sl = slice(h * n, (h + 1) * n)
        dT = torch.from_numpy(np.ascontiguousarray(T[:, sl])).cuda()
        got, gn = ctx.chain_poses(dT, torch.from_numpy(np.ascontiguousarray(St[:, sl])).cuda(), cum,
                                  n_points=torch.from_numpy(np.ascontiguousarray(N[:, sl])).cuda())
        want, wn, ref_cum = _chain_ref(T[:, sl], St[:, sl], N[:, sl], ref_cum)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy(), want) and np.array_equal(gn.cpu().numpy(), wn)
    assert np.array_equal(cum.cpu().numpy(), ref_cum)
    for s in range(S_):
        posed = St[s] >= 0
        assert np.allclose(ev.chain(T[s], posed)[-1], ref_cum[s], rtol=0, atol=1e-12)
