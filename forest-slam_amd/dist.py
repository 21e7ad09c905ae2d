"""Multi-GPU sharding of the VO path: one process per GPU.

* Sequence-per-GPU (configs 4/5): rank r processes sequences r, r+N, ... independently;
  no data-path collective.  ``sequences_for_rank``.
* Frame-pair sharding inside ONE sequence: frame pairs are independent;
  rank r processes pairs [s_r, e_r) reading images [s_r - 1, e_r) (one-image halo), then
  the relative poses are exchanged with one all-gather and every rank composes the chain
  left to right in float64 — bit-identical to the single-GPU chain (stereo_slam.py:306).
  ``frame_shard`` / ``gather_relative_poses``.
* Keyframe exchange for the multi-sequence map: ``allgather_keyframes`` (poses + landmark
  positions, tens of KB: latency-bound, one collective per window step).

Collectives go through ``torch.distributed`` (backend "nccl" = RCCL over xGMI on the
MI355X node; "gloo" in the CPU tests).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def sequences_for_rank(rank: int, world: int, n_sequences: int) -> list[int]:
    return list(range(rank, n_sequences, world))


def frame_shard(n_pairs: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [start, end) of the frame-pair indices 1..n_pairs (pair i uses
    images i-1 and i), balanced to within one pair."""
    q, r = divmod(n_pairs, world)
    start = rank * q + min(rank, r)
    end = start + q + (1 if rank < r else 0)
    return 1 + start, 1 + end


def gather_relative_poses(T_local: torch.Tensor, status_local: torch.Tensor, n_pairs: int,
                          group=None) -> tuple[np.ndarray, np.ndarray]:
    """All-gather every rank's relative transforms (f64 [n_r,4,4]) and statuses into the
    full per-pair arrays (rank order == frame order)."""
    world = dist.get_world_size(group)
    dev = T_local.device
    counts = [frame_shard(n_pairs, r, world) for r in range(world)]
    maxn = max(e - s for s, e in counts)
    padT = torch.zeros((maxn, 4, 4), dtype=torch.float64, device=dev)
    padS = torch.full((maxn,), -2, dtype=torch.int32, device=dev)
    padT[:T_local.shape[0]] = T_local
    padS[:status_local.shape[0]] = status_local
    outT = [torch.empty_like(padT) for _ in range(world)]
    outS = [torch.empty_like(padS) for _ in range(world)]
    dist.all_gather(outT, padT, group=group)
    dist.all_gather(outS, padS, group=group)
    T = np.concatenate([outT[r][:e - s].cpu().numpy() for r, (s, e) in enumerate(counts)])
    S = np.concatenate([outS[r][:e - s].cpu().numpy() for r, (s, e) in enumerate(counts)])
    return T, S


def exchange_window_map(T_step: torch.Tensor, lm_xyz: torch.Tensor, lm_count: torch.Tensor, group=None):
    """The per-step map exchange of the multi-sequence run: every rank's
    BA-refined relative poses of the step (f64 [B,4,4]) and its latest window's landmarks
    (f64 [Lmax,3] + i32 [1] count, fixed size) are all-gathered over RCCL.  Fixed shapes and
    device-side counts: no host synchronisation, the collectives queue behind the step's
    kernels.  Returns (T [world,B,4,4], xyz [world,Lmax,3], counts [world,1])."""
    world = dist.get_world_size(group)
    outT = [torch.empty_like(T_step) for _ in range(world)]
    outX = [torch.empty_like(lm_xyz) for _ in range(world)]
    outC = [torch.empty_like(lm_count) for _ in range(world)]
    dist.all_gather(outT, T_step.contiguous(), group=group)
    dist.all_gather(outX, lm_xyz.contiguous(), group=group)
    dist.all_gather(outC, lm_count.contiguous(), group=group)
    return torch.stack(outT), torch.stack(outX), torch.stack(outC)


def allgather_keyframes(poses: torch.Tensor, landmarks: torch.Tensor, group=None):
    """Exchange each rank's window keyframe poses (f32 [K,7]) and active landmarks
    (f32 [L_r,3], variable L_r) -> lists indexed by rank."""
    world = dist.get_world_size(group)
    dev = poses.device
    n = torch.tensor([landmarks.shape[0]], dtype=torch.int64, device=dev)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    maxl = int(max(int(x.item()) for x in ns))
    pad = torch.zeros((max(maxl, 1), 3), dtype=landmarks.dtype, device=dev)
    pad[:landmarks.shape[0]] = landmarks
    outp = [torch.empty_like(poses) for _ in range(world)]
    outl = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outp, poses.contiguous(), group=group)
    dist.all_gather(outl, pad, group=group)
    return outp, [outl[r][:int(ns[r].item())] for r in range(world)]
