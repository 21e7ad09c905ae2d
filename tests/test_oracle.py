"""CPU tests of the oracle (test infrastructure): golden vectors, independent brute-force
cross-checks of the restated OpenCV semantics, and known-answer tests."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "golden_small.npz"))


def test_golden_vectors_reproduce(oracle_mod, golden):
    g = golden
    kp0, d0 = oracle_mod.orb_detect_compute(g["L0"], 300)
    kp1, d1 = oracle_mod.orb_detect_compute(g["L1"], 300)
    assert np.array_equal(kp0, g["kp0"]) and np.array_equal(d0, g["d0"])
    assert np.array_equal(kp1, g["kp1"]) and np.array_equal(d1, g["d1"])
    m = oracle_mod.bf_match(d0, d1)
    assert np.array_equal(m, g["matches"])
    disp = oracle_mod.sgbm(g["L0"], g["R0"], num_disp=64)
    assert np.array_equal(disp, g["disp16"])
    mk0 = kp0[:, :2].astype(np.float32)[m[:, 0]]
    mk1 = kp1[:, :2].astype(np.float32)[m[:, 1]]
    P3, p2, _ = oracle_mod.backproject(oracle_mod.disparity_map(disp), mk0, mk1, g["K"], 0.253736175410149)
    assert np.array_equal(P3, g["P3"]) and np.array_equal(p2, g["p2"])
    from forest_slam_amd import synth
    ok, rv, tv, inl, ni, _ = oracle_mod.solve_pnp_ransac(P3, p2, g["K"], synth.DIST_L)
    assert ok == bool(g["pnp_ok"]) and ni == int(g["ransac_iters"])
    assert np.array_equal(inl, g["inliers"])
    assert np.allclose(rv, g["rvec"], rtol=0, atol=1e-12) and np.allclose(tv, g["tvec"], rtol=0, atol=1e-12)


def test_orb_level_geometry_and_budgets(oracle_mod):
    """SURVEY.md §8 header: level sizes and per-level feature budgets."""
    img = np.zeros((600, 960), np.uint8)
    sizes = [lv.shape[::-1] for lv in oracle_mod.orb_pyramid(img, 8)]
    assert sizes == [(960, 600), (800, 500), (667, 417), (556, 347), (463, 289), (386, 241), (322, 201), (268, 167)]
    assert list(oracle_mod.features_per_level(500)) == [109, 90, 75, 63, 52, 44, 36, 31]
    assert list(oracle_mod.features_per_level(1000)) == [217, 181, 151, 126, 105, 87, 73, 60]
    assert list(oracle_mod.features_per_level(2000)) == [434, 362, 302, 251, 209, 175, 145, 122]


def _fast_brute(img, t):
    """Independent pure-Python FAST-9/16 + cornerScore (definition form)."""
    circ = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2), (-3, -1),
            (-3, 0), (-3, 1), (-2, 2), (-1, 3)]
    H, W = img.shape
    out = np.zeros((H, W), np.uint8)
    for y in range(3, H - 3):
        for x in range(3, W - 3):
            v = int(img[y, x])
            p = [int(img[y + dy, x + dx]) for dx, dy in circ]
            br = [q > v + t for q in p]
            dk = [q < v - t for q in p]
            def arc(m):
                return any(all(m[(s + j) % 16] for j in range(9)) for s in range(16))
            if arc(br) or arc(dk):
                best = t
                for s in range(16):
                    d = [v - p[(s + j) % 16] for j in range(9)]
                    best = max(best, min(d), min(-q for q in d))
                out[y, x] = best - 1
    return out


def test_fast_score_matches_definition(oracle_mod):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (40, 48)).astype(np.uint8)
    img[10:20, 10:20] = 250
    for t in (10, 20, 40):
        assert np.array_equal(oracle_mod.fast_score_map(img, t), _fast_brute(img, t))


def test_fast_nms_row_major(oracle_mod):
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (64, 80)).astype(np.uint8)
    s = oracle_mod.fast_score_map(img, 20).astype(int)
    kp = oracle_mod.fast_detect(img, 20)
    want = []
    for y in range(3, 61):
        for x in range(3, 77):
            c = s[y, x]
            if c and all(c > s[y + dy, x + dx] for dy in (-1, 0, 1) for dx in (-1, 0, 1) if dy or dx):
                want.append((x, y, c))
    assert [tuple(r) for r in kp] == want


def test_retain_best_keeps_top_and_ties(oracle_mod):
    rng = np.random.default_rng(5)
    for n, keep in [(100, 10), (1000, 434), (57, 57), (20, 30)]:
        r = rng.integers(0, 12, n).astype(np.float32)
        idx = oracle_mod.retain_best(r, keep)
        if keep >= n:
            assert np.array_equal(idx, np.arange(n))
            continue
        b = np.sort(r)[::-1][keep - 1]
        assert set(idx.tolist()) == set(np.nonzero(r >= b)[0].tolist())


def test_bf_match_brute_force(oracle_mod):
    rng = np.random.default_rng(6)
    d0 = rng.integers(0, 256, (120, 32)).astype(np.uint8)
    d1 = np.concatenate([d0[::2] ^ (rng.random((60, 32)) < 0.02).astype(np.uint8), rng.integers(0, 256, (40, 32)).astype(np.uint8)])
    bits = lambda a, b: np.unpackbits(a[:, None, :] ^ b[None, :, :], axis=2).sum(2)  # noqa: E731
    D = bits(d0, d1)
    s = D.argmin(1)  # argmin -> first index on ties, as OpenCV
    t = D.argmin(0)
    want = [(q, s[q], D[q, s[q]]) for q in range(len(d0)) if t[s[q]] == q]
    got = oracle_mod.bf_match(d0, d1)
    assert [tuple(r) for r in got] == want


def test_fast_atan2_accuracy(oracle_mod):
    for y, x in [(1, 0), (0, 1), (-1, -1), (3, -4), (-2, 5), (100, 1), (0, -1)]:
        a = oracle_mod.fast_atan2(y, x)
        ref = np.degrees(np.arctan2(y, x)) % 360
        assert abs(((a - ref) + 180) % 360 - 180) < 0.02


def test_sgbm_recovers_synthetic_disparity(oracle_mod):
    """Shifted random texture: the disparity equals the shift (x16) away from borders."""
    rng = np.random.default_rng(7)
    base = (rng.random((120, 300)) * 255).astype(np.uint8)
    L = base[:, 20:260].copy()
    R = base[:, 20 + 13:260 + 13].copy()  # right view sees scene shifted: disparity 13 at every pixel
    # right image pixel x corresponds to left x - d -> R[x] = L[x + d]
    R = np.roll(L, 0, axis=1)
    R[:, :-13] = L[:, 13:]
    d = oracle_mod.sgbm(L, R, num_disp=64)
    core = d[10:-10, 80:-10]
    assert np.median(core) == 13 * 16
    assert np.mean(np.abs(core.astype(int) - 208) <= 8) > 0.95
    assert (d[:, :64] == -16).all()  # OpenCV leaves the first numDisparities columns invalid


def test_pnp_known_answer(oracle_mod):
    from forest_slam_amd import synth
    rng = np.random.default_rng(8)
    n = 200
    P = np.c_[rng.uniform(-5, 5, n), rng.uniform(-2, 2, n), rng.uniform(3, 30, n)].astype(np.float32).astype(np.float64)
    rv = np.array([0.01, -0.02, 0.005])
    tv = np.array([0.05, -0.01, 0.12])
    uv = oracle_mod.project_points(P, rv, tv, synth.K0, synth.DIST_L)
    ok, r, t, inl, _, _ = oracle_mod.solve_pnp_ransac(P, uv.astype(np.float32), synth.K0, synth.DIST_L)
    assert ok and len(inl) == n
    assert np.abs(r - rv).max() < 1e-6 and np.abs(t - tv).max() < 1e-6


def test_rodrigues_roundtrip(oracle_mod):
    from scipy.spatial.transform import Rotation
    for rv in [np.array([0.3, -0.2, 0.1]), np.array([1e-9, 0, 0]), np.array([0.0, 3.0, 0.1])]:
        R = oracle_mod.rodrigues(rv)
        assert np.allclose(R, Rotation.from_rotvec(rv).as_matrix(), atol=1e-12)


def test_backproject_numpy1_semantics(oracle_mod):
    """float32 arithmetic with float64 scalars rounded first (NumPy 1.x value-based casting)."""
    disp = np.array([[0, -16, 32, 160]], np.int16)
    d = oracle_mod.disparity_map(disp)
    assert d.dtype == np.float32 and d[0, 0] == np.float32(0.1) and d[0, 1] == np.float32(0.1)
    K = np.array([[642.9165664800531, 0, 460.1840658156501], [0, 641.9171825800378, 308.584644910031], [0, 0, 1]])
    mk = np.array([[2.4, 0.2], [3.9, 0.7], [1.0, 0.0]], np.float32)
    P, p2, valid = oracle_mod.backproject(d, mk, mk, K, 0.253736175410149)
    assert P.dtype == np.float32
    Z = np.float32(K[0, 0] * 0.253736175410149) / d[0, [2, 3, 1]]
    assert valid.tolist() == [bool(z > np.float32(0.1) and z < 1000) for z in Z]
