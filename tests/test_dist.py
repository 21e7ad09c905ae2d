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
    Tw, Sw, Xw, Cw = fd.exchange_window_map(torch.full((4, 4, 4), float(rank), dtype=torch.float64),
                                            torch.full((4,), rank - 1, dtype=torch.int32),
                                            torch.full((16, 3), 10.0 + rank, dtype=torch.float64),
                                        torch.tensor([rank + 5], dtype=torch.int32))
    out[rank] = (T, S, [p[0, 0].item() for p in poses], [l.shape[0] for l in lms],
                 (Tw[:, 0, 0, 0].tolist(), Xw[:, 0, 0].tolist(), Cw[:, 0].tolist(), Sw[:, 3].tolist()))
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
        T, S, kf, nl, wm = out[r]
        assert wm == ([0.0, 1.0], [10.0, 11.0], [5, 6], [-1, 0])
        assert np.array_equal(T, allT)
        assert S[3] == -1 and (S[np.arange(n_pairs) != 3] == 1).all()
        assert kf == [0.0, 1.0] and nl == [2, 3]
        # chaining the gathered poses equals the single-process chain exactly
        assert np.array_equal(ev.chain(T, S != -1), ev.chain(allT, S != -1))


def test_map_chain_places_landmarks_with_the_reference_chain():
    """dist.MapChain (GlobalMap's host side): per rank the gathered relative poses chained as
    eval.chain does (status -1 / overflow frames keep the pose), and each step's landmarks
    placed with the chain through s+1, s = the first frame of the step's last BA window."""
    from forest_slam_amd import dist as fd
    from forest_slam_amd import eval as ev
    rng = np.random.default_rng(5)
    world, K, B, steps = 3, 4, 3, 4
    T = np.tile(np.eye(4), (world, B * steps, 1, 1))
    T[..., :3, 3] = rng.normal(0, 0.3, (world, B * steps, 3))
    S = np.ones((world, B * steps), np.int32)
    S[1, 4] = -1
    S[2, 7] = -3
    mc = fd.MapChain(world, K)
    got = [mc.advance(T[:, k * B:(k + 1) * B], S[:, k * B:(k + 1) * B]) for k in range(steps)]
    for r in range(world):
        valid = (S[r] != -1) & (S[r] != -3)
        cum = ev.chain(T[r], valid)  # TUM chain: the poses of the valid frames
        full = [np.eye(4)]
        j = 0
        for f in range(B * steps):
            if valid[f]:
                full.append(cum[j])
                j += 1
            else:
                full.append(full[-1])
        for k in range(steps):
            e = (k + 1) * B
            s = max(0, e - K + 1)
            assert np.array_equal(got[k][r], full[s + 1]), (r, k)
