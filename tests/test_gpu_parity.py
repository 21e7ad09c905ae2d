"""GPU parity: every HIP stage vs the oracle (bit-exact for integer/byte/index work).

Runs on the MI355X box (``pytest -m gpu``).  Inputs are seeded synthetic forest frames
(rendered on the CPU so both sides see identical bytes) plus adversarial arrays.
"""
import numpy as np
import pytest
import torch

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]


@pytest.fixture(scope="module")
def frames():
    import forest_slam_amd.synth as synth
    seq = synth.StereoSequence(seed=3, n_frames=4, W=960, H=600, device="cpu")
    out = [seq.frame(i) for i in range(3)]
    return [(L.numpy(), R.numpy()) for L, R in out]


@pytest.fixture(scope="module")
def ctx600():
    from forest_slam_amd import _lib
    return _lib.Context(960, 600, max_batch=4, nfeatures=500)


def _orb_gpu(ctx, imgs):
    t = torch.from_numpy(np.stack(imgs)).cuda()
    kp, desc, cnt = ctx.orb(t)
    torch.cuda.synchronize()
    cnt = cnt.cpu().numpy()
    return [(kp[i, :cnt[i]].cpu().numpy(), desc[i, :cnt[i]].cpu().numpy()) for i in range(len(imgs))], cnt


def test_retain_best_matches_libstdcxx(oracle_mod):
    from forest_slam_amd import _lib
    ctx = _lib.Context(128, 128, max_batch=1)
    rng = np.random.default_rng(0)
    cases = []
    for n in [1, 2, 3, 4, 5, 7, 16, 33, 100, 513, 1000, 4097, 20000]:
        for keep in sorted({1, 2, 3, max(1, n // 7), max(1, n // 2), max(1, n - 1), n, n + 5}):
            cases.append((n, keep, "ties"))
            cases.append((n, keep, "uniform"))
    for n, keep, kind in cases:
        if kind == "ties":
            keys = rng.integers(19, 40, size=n).astype(np.float32)
        else:
            keys = rng.standard_normal(n).astype(np.float32)
        want = oracle_mod.retain_best(keys, keep)
        got = ctx.test_retain_best(torch.from_numpy(keys), keep).cpu().numpy()
        assert np.array_equal(got, want), (n, keep, kind)
    # sorted / reversed / constant inputs (median-of-3 edge cases)
    for keys in [np.arange(3000, dtype=np.float32), np.arange(3000, 0, -1).astype(np.float32),
                 np.full(3000, 7.0, np.float32), np.tile(np.arange(5, dtype=np.float32), 800)]:
        for keep in [1, 10, 999, 2999]:
            want = oracle_mod.retain_best(keys, keep)
            got = ctx.test_retain_best(torch.from_numpy(keys), keep).cpu().numpy()
            assert np.array_equal(got, want)


def test_pyramid_and_fast_bit_exact(oracle_mod, ctx600, frames):
    L = frames[0][0]
    _orb_gpu(ctx600, [L])
    geo, total = ctx600.geometry()
    pyr = ctx600.debug_buffer(0).numpy()[:total]
    ref_levels = oracle_mod.orb_pyramid(L, 8)
    for (w, h, off), ref in zip(geo, ref_levels):
        got = pyr[off:off + w * h].reshape(h, w)
        assert got.shape == ref.shape
        assert np.array_equal(got, ref), f"pyramid level {w}x{h} differs at {np.argwhere(got != ref)[:5]}"
    score = ctx600.debug_buffer(2).numpy()[:total]
    for (w, h, off), lvl in zip(geo, ref_levels):
        ref = oracle_mod.fast_score_map(lvl, 20)
        got = score[off:off + w * h].reshape(h, w)
        assert np.array_equal(got, ref), f"FAST score {w}x{h}: {np.argwhere(got != ref)[:5]}"
    blur = ctx600.debug_buffer(1).numpy()[:total]
    ref_b = oracle_mod.orb_pyramid(L, 8, blurred=True)
    for (w, h, off), ref in zip(geo, ref_b):
        assert np.array_equal(blur[off:off + w * h].reshape(h, w), ref)


@pytest.mark.parametrize("nfeatures", [500, 1000])
def test_orb_bit_exact(oracle_mod, frames, nfeatures):
    from forest_slam_amd import _lib
    ctx = _lib.Context(960, 600, max_batch=4, nfeatures=nfeatures)
    imgs = [frames[0][0], frames[0][1], frames[1][0], frames[2][0]]
    got, cnt = _orb_gpu(ctx, imgs)
    for img, (kp, desc) in zip(imgs, got):
        rkp, rdesc = oracle_mod.orb_detect_compute(img, nfeatures)
        assert kp.shape[0] == rkp.shape[0]
        assert np.array_equal(kp[:, :6], rkp), np.argwhere(kp[:, :6] != rkp)[:5]
        assert np.array_equal(desc, rdesc)


def test_bf_match_bit_exact(oracle_mod, frames):
    from forest_slam_amd import _lib
    ctx = _lib.Context(960, 600, max_batch=3, nfeatures=1000)
    _, d0 = oracle_mod.orb_detect_compute(frames[0][0], 1000)
    _, d1 = oracle_mod.orb_detect_compute(frames[1][0], 1000)
    rng = np.random.default_rng(1)
    # adversarial: few distinct descriptors -> many distance ties
    base = rng.integers(0, 256, size=(8, 32), dtype=np.uint8)
    r0 = base[rng.integers(0, 8, 700)]
    r1 = base[rng.integers(0, 8, 650)]
    r1[::3, 0] ^= 1
    sets = [(d0, d1), (r0, r1), (d0[:1], d1)]
    cap = ctx.kp_cap
    Q = np.zeros((3, cap, 32), np.uint8)
    T = np.zeros((3, cap, 32), np.uint8)
    nq = np.zeros(3, np.int32)
    nt = np.zeros(3, np.int32)
    for i, (a, b) in enumerate(sets):
        Q[i, :len(a)] = a
        T[i, :len(b)] = b
        nq[i], nt[i] = len(a), len(b)
    m, nm = ctx.bf_match(torch.from_numpy(Q).cuda(), torch.from_numpy(nq).cuda(), torch.from_numpy(T).cuda(),
                         torch.from_numpy(nt).cuda())
    torch.cuda.synchronize()
    m, nm = m.cpu().numpy(), nm.cpu().numpy()
    for i, (a, b) in enumerate(sets):
        want = oracle_mod.bf_match(a, b)
        assert nm[i] == len(want)
        assert np.array_equal(m[i, :nm[i]], want)


def test_sgbm_bit_exact(oracle_mod, frames):
    from forest_slam_amd import _lib
    ctx = _lib.Context(960, 600, max_batch=2)
    L = np.stack([frames[0][0], frames[1][0]])
    R = np.stack([frames[0][1], frames[1][1]])
    d = ctx.sgbm(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda())
    torch.cuda.synchronize()
    d = d.cpu().numpy()
    for i in range(2):
        want = oracle_mod.sgbm(L[i], R[i])
        bad = np.argwhere(d[i] != want)
        assert len(bad) == 0, f"pair {i}: {len(bad)} px differ, first {bad[:5]}"


def test_sgbm_small_geometry(oracle_mod):
    """Non-default geometry: 320x200, 64 disparities, stripes of 50 rows."""
    from forest_slam_amd import _lib
    import forest_slam_amd.synth as synth
    seq = synth.StereoSequence(seed=5, n_frames=2, W=320, H=200, device="cpu")
    L, R = seq.frame(1)
    ctx = _lib.Context(320, 200, max_batch=1, num_disparities=64)
    d = ctx.sgbm(L.cuda(), R.cuda())
    torch.cuda.synchronize()
    want = oracle_mod.sgbm(L.numpy(), R.numpy(), num_disp=64)
    assert np.array_equal(d[0].cpu().numpy(), want)
