"""Natural-image parity (VERDICT r1 "real-image fixtures"): scikit-image's camera / grass /
gravel / brick and their 960x600 montage for ORB at 500 and 1000 features, the rectified
Middlebury motorcycle pair for SGBM (96 and 128 disparities) and BF.  Fixtures and the
oracle digests: tests/golden/make_golden_natural.py.

CPU: the oracle reproduces the committed digests, and its SGBM agrees with the Middlebury
ground truth (a semantic check that the restated algorithm is a working SGBM-3way).
GPU: the HIP path equals the oracle bit for bit on every fixture."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, gpu_available


@pytest.fixture(scope="module")
def nat():
    z = np.load(os.path.join(GOLDEN, "natural_images.npz"))
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def digests():
    with open(os.path.join(GOLDEN, "natural_oracle.json")) as f:
        return json.load(f)


def _gen():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden_natural", os.path.join(GOLDEN, "make_golden_natural.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


ORB_IMAGES = ("camera", "grass", "gravel", "brick", "montage600")


def test_oracle_reproduces_natural_digests(oracle_mod, nat, digests):
    got = _gen().oracle_outputs(nat)
    assert got == digests


def test_oracle_sgbm_agrees_with_middlebury_ground_truth(oracle_mod, nat):
    gt = nat["moto_gt16"].astype(np.float64) / 16
    d = oracle_mod.sgbm(nat["moto_L"], nat["moto_R"]).astype(np.float64) / 16
    ok = (gt > 0) & (d >= 0)
    err = np.abs(d - gt)[ok]
    assert ok.sum() > 0.8 * (gt > 0).sum()
    assert (err < 1).mean() > 0.88 and (err < 2).mean() > 0.9


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
@pytest.mark.parametrize("nfeatures", [500, 1000])
def test_gpu_orb_natural_bit_exact(oracle_mod, nat, digests, nfeatures):
    from forest_slam_amd import _lib
    gen = _gen()
    ctx512 = _lib.Context(512, 512, max_batch=4, nfeatures=nfeatures)
    ctx600 = _lib.Context(960, 600, max_batch=1, nfeatures=nfeatures)
    for ctx, names in ((ctx512, ORB_IMAGES[:4]), (ctx600, ORB_IMAGES[4:])):
        imgs = torch.from_numpy(np.stack([nat[n] for n in names])).cuda()
        kp, desc, cnt = ctx.orb(imgs)
        torch.cuda.synchronize()
        for i, name in enumerate(names):
            c = int(cnt[i].item())
            k = kp[i, :c, :6].cpu().numpy()
            d = desc[i, :c].cpu().numpy()
            rk, rd = oracle_mod.orb_detect_compute(nat[name], nfeatures)
            assert c == len(rk), (name, c, len(rk))
            assert np.array_equal(k, rk), (name, np.argwhere(k != rk)[:4])
            assert np.array_equal(d, rd), name
            assert gen.digest(rk, rd) == digests[f"orb/{name}/{nfeatures}"]["sha256"]


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
@pytest.mark.parametrize("ndisp", [96, 128])
def test_gpu_sgbm_middlebury_bit_exact(oracle_mod, nat, ndisp):
    from forest_slam_amd import _lib
    L, R = nat["moto_L"], nat["moto_R"]
    H, W = L.shape
    ctx = _lib.Context(W, H, max_batch=1, num_disparities=ndisp)
    d = ctx.sgbm(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda())
    torch.cuda.synchronize()
    d = d[0].cpu().numpy()
    want = oracle_mod.sgbm(L, R, num_disp=ndisp)
    bad = np.argwhere(d != want)
    assert len(bad) == 0, f"{len(bad)} px differ, first {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")
def test_gpu_bf_middlebury_bit_exact(oracle_mod, nat):
    from forest_slam_amd import _lib
    L, R = nat["moto_L"], nat["moto_R"]
    H, W = L.shape
    ctx = _lib.Context(W, H, max_batch=2, nfeatures=1000)
    kp, desc, cnt = ctx.orb(torch.from_numpy(np.stack([L, R])).cuda())
    m, nm = ctx.bf_match(desc[0:1], cnt[0:1], desc[1:2], cnt[1:2])
    torch.cuda.synchronize()
    _, d0 = oracle_mod.orb_detect_compute(L, 1000)
    _, d1 = oracle_mod.orb_detect_compute(R, 1000)
    want = oracle_mod.bf_match(d0, d1)
    assert int(nm[0].item()) == len(want)
    assert np.array_equal(m[0, :len(want)].cpu().numpy(), want)
