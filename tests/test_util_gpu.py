"""Step bookkeeping entry points (fvo_copy_regions, fvo_count_guard) against torch on the GPU.

They replace torch copies / elementwise ops in the front end's step (vo.StereoFrontEnd), so the
reference is plain torch on the same tensors; every byte must match."""
import pytest
import torch

from forest_slam_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return _lib.Context(64, 64, max_batch=2, device=torch.device("cuda", 0), stages=_lib.STAGE_ORB)


def test_copy_regions_matches_torch_copies(ctx):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(3)
    srcs, dsts, pairs = [], [], []
    # 16-B, 4-B and 1-B aligned regions, empty ones, one region larger than a block's sweep
    for nbytes, off in [(4096, 0), (1 << 20, 16), (1028, 4), (999, 1), (0, 0), (7, 3), (3 << 20, 0)]:
        s = torch.randint(0, 256, (nbytes + 32,), dtype=torch.uint8, generator=g).to(dev)
        d = torch.zeros(nbytes + 32, dtype=torch.uint8, device=dev)
        srcs.append(s)
        dsts.append(d)
        pairs.append((d[off:off + nbytes], s[off:off + nbytes]))
    ctx.copy_regions(pairs)
    torch.cuda.synchronize()
    for (d, s), full in zip(pairs, dsts):
        assert torch.equal(d, s)
    # bytes outside the regions untouched
    for (nbytes, off), full in zip([(4096, 0), (1 << 20, 16), (1028, 4), (999, 1), (0, 0), (7, 3), (3 << 20, 0)], dsts):
        assert int(full[:off].count_nonzero()) == 0 and int(full[off + nbytes:].count_nonzero()) == 0


def test_copy_regions_typed_slices_and_many_regions(ctx):
    dev = torch.device("cuda", 0)
    a = torch.randn(40, 17, 8, device=dev)
    b = torch.zeros_like(a)
    c = torch.arange(100, dtype=torch.int32, device=dev)
    d = torch.zeros(100, dtype=torch.int32, device=dev)
    pairs = [(b[i], a[39 - i]) for i in range(40)] + [(d[10:60], c[40:90])]  # > FVO_MAX_REGIONS: two launches
    ctx.copy_regions(pairs)
    torch.cuda.synchronize()
    assert torch.equal(b, a.flip(0))
    assert torch.equal(d[10:60], c[40:90]) and int(d[:10].count_nonzero()) == 0


def test_copy_regions_refuses_overlap(ctx):
    x = torch.arange(64, dtype=torch.int32, device=torch.device("cuda", 0))
    with pytest.raises(RuntimeError, match="overlap"):
        ctx.copy_regions([(x[0:32], x[16:48])])
    with pytest.raises(RuntimeError, match="overlap"):
        ctx.copy_regions([(x[0:8], x[32:40]), (x[4:12], x[48:56])])


@pytest.mark.parametrize("sets,with_q", [(1, True), (2, True), (2, False), (1, False)])
def test_count_guard_matches_torch(ctx, sets, with_q):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(sets * 7 + with_q)
    n = 300
    cnt = torch.randint(-5, 50, (sets * n,), dtype=torch.int32, generator=g).to(dev)
    q = torch.randint(-5, 50, (sets * n,), dtype=torch.int32, generator=g).to(dev) if with_q else None
    st = torch.randint(-1, 2, (n,), dtype=torch.int32, generator=g).to(dev)
    st_ref = st.clone()
    clamped = torch.full((n,), 77, dtype=torch.int32, device=dev)
    ctx.count_guard(cnt, n, sets, q_counts=q, status=st, code=-3, clamped_out=clamped)
    over = torch.zeros(n, dtype=torch.bool, device=dev)
    for s in range(sets):
        over |= cnt[s * n:(s + 1) * n] < 0
        if with_q:
            over |= q[s * n:(s + 1) * n] < 0
    st_ref.masked_fill_(over, -3)
    torch.cuda.synchronize()
    assert torch.equal(st, st_ref)
    assert torch.equal(clamped, cnt[:n].clamp(min=0))
