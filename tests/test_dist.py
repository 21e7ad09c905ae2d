"""Multi-process (world_size 2, gloo on CPU) tests of the sharding helpers."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_pairs, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    from forest_slam_amd import dist as fd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(0)
    allT = np.tile(np.eye(4), (n_pairs, 1, 1))
    allT[:, :3, 3] = rng.normal(0, 0.1, (n_pairs, 3))
    allS = np.ones(n_pairs, np.int32)
    allS[3] = -1
    s, e = fd.frame_shard(n_pairs, rank, world)
    T, S = fd.gather_relative_poses(torch.from_numpy(allT[s - 1:e - 1]), torch.from_numpy(allS[s - 1:e - 1]), n_pairs)
    poses, lms = fd.allgather_keyframes(torch.full((10, 7), float(rank)), torch.ones((rank + 2, 3)) * rank)
    Tw, Sw, Pw, Nw = fd.exchange_frame_map(torch.full((4, 4, 4), float(rank), dtype=torch.float64),
                                           torch.full((4,), rank - 1, dtype=torch.int32),
                                           torch.full((4, 16, 3), 10.0 + rank, dtype=torch.float32),
                                           torch.tensor([rank + 5, 1, 2, 3], dtype=torch.int32))
    g0 = fd.exchange_frame_map(torch.full((4, 4, 4), float(rank), dtype=torch.float64),
                               torch.full((4,), rank - 1, dtype=torch.int32),
                               torch.full((4, 16, 3), 10.0 + rank, dtype=torch.float32),
                               torch.tensor([rank + 5, 1, 2, 3], dtype=torch.int32), dst=0)  # map on rank 0 only
    g0 = None if g0 is None else (g0[0][:, 0, 0, 0].tolist(), g0[2][:, 0, 0, 0].tolist(), g0[3][:, 0].tolist())
    out[rank] = (T, S, [p[0, 0].item() for p in poses], [l.shape[0] for l in lms],
                 (Tw[:, 0, 0, 0].tolist(), Pw[:, 0, 0, 0].tolist(), Nw[:, 0].tolist(), Sw[:, 3].tolist()), g0)
    dist.barrier()
    dist.destroy_process_group()


def test_frame_shards_cover_sequence():
    from forest_slam_amd import dist as fd
    for n in (1, 7, 962):
        for w in (1, 2, 3, 8):
            spans = [fd.frame_shard(n, r, w) for r in range(w)]
            assert spans[0][0] == 1 and spans[-1][1] == n + 1
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert fd.sequences_for_rank(1, 4, 8) == [1, 5]


def test_gather_poses_two_ranks_gloo():
    from forest_slam_amd import eval as ev
    n_pairs = 11
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.spawn(_worker, args=(2, port, n_pairs, out), nprocs=2, join=True)
    rng = np.random.default_rng(0)
    allT = np.tile(np.eye(4), (n_pairs, 1, 1))
    allT[:, :3, 3] = rng.normal(0, 0.1, (n_pairs, 3))
    for r in range(2):
        T, S, kf, nl, wm, g0 = out[r]
        assert wm == ([0.0, 1.0], [10.0, 11.0], [5, 6], [-1, 0])
        assert g0 == (([0.0, 1.0], [10.0, 11.0], [5, 6]) if r == 0 else None)  # gathered to rank 0 only
        assert np.array_equal(T, allT)
        assert S[3] == -1 and (S[np.arange(n_pairs) != 3] == 1).all()
        assert kf == [0.0, 1.0] and nl == [2, 3]
        # chaining the gathered poses equals the single-process chain exactly
        assert np.array_equal(ev.chain(T, S != -1), ev.chain(allT, S != -1))


class _FakeFrontEnd:
    """CPU stand-in for vo.StereoFrontEnd: pair i -> a translation of i (image values carry i)."""
    B, ba_window = 4, 3

    def prime(self, L, R):
        self.prev = float(L[0, 0])

    def step(self, L, R):
        n = L.shape[0]
        T = torch.eye(4, dtype=torch.float64).repeat(n, 1, 1)
        T[:, 0, 3] = L[:, 0, 0].double()
        self.T = T
        return T, torch.ones(n, dtype=torch.int32)


def test_run_sequence_sharded_without_process_group():
    """bench.py --shard frames --gpus 1 starts no process group: the sharded run is the whole
    sequence on one rank (it raised 'Default process group has not been initialized')."""
    import torch.distributed as dist
    from forest_slam_amd import dist as fd
    from forest_slam_amd import eval as ev
    assert not dist.is_initialized()
    n_img = 11
    imgs = torch.arange(n_img, dtype=torch.uint8)[:, None, None].expand(n_img, 2, 2).contiguous()
    rows, T, S = fd.run_sequence_sharded(_FakeFrontEnd, imgs, imgs)
    assert T.shape == (n_img - 1, 4, 4) and (S == 1).all()
    assert np.array_equal(T[:, 0, 3], np.arange(1, n_img, dtype=np.float64))
    assert np.array_equal(rows[:, 1], ev.chain(T, S != -1)[:, 0, 3])
