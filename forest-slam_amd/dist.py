"""Multi-GPU sharding of the VO path: one process per GPU.

* Sequence-per-GPU (configs 4/5): rank r processes sequences r, r+N, ... independently;
  no data-path collective.  ``sequences_for_rank``.
* Frame-pair sharding inside ONE sequence: frame pairs are independent;
  rank r processes pairs [s_r, e_r) reading images [s_r - 1, e_r) (one-image halo), then
  the relative poses are exchanged with one all-gather and every rank composes the chain
  left to right in float64.  For the PnP-only path (ba_window = 0) this is bit-identical to
  the single-GPU chain (stereo_slam.py:306).  With local BA a window needs the K-1 frames
  before its last one: ``frame_shard(..., halo=K-1)`` starts the rank's front end K-1 images
  earlier and ``warmup_pairs`` of its first results (the windows that reach back past the
  shard start on one GPU but not here) are discarded — the previous rank owns those pairs.
  ``frame_shard`` / ``gather_relative_poses``; ``run_sequence_sharded`` is the whole
  single-sequence run (bench.py --shard frames).
* ``SequenceRank`` — one rank's step of the multi-sequence run (bench.py, tests): the
  front-end step, then on a side stream the map exchange of the step's poses and every
  frame's points3D (``exchange_frame_map``) and the multi-sequence map built from it on the
  device (``GlobalMap``: ``fvo_chain_poses`` + ``fvo_map_transform``).
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


def frame_shard(n_pairs: int, rank: int, world: int, halo: int = 0) -> tuple[int, int]:
    """Contiguous shard [start, end) of the frame-pair indices 1..n_pairs (pair i uses
    images i-1 and i), balanced to within one pair.  ``halo`` > 0 (local BA: K-1) moves the
    start back by up to that many pairs; the caller drops the first ``start_owned - start``
    results (``warmup_pairs``)."""
    q, r = divmod(n_pairs, world)
    start = rank * q + min(rank, r)
    end = start + q + (1 if rank < r else 0)
    return 1 + max(0, start - halo), 1 + end


def warmup_pairs(n_pairs: int, rank: int, world: int, halo: int) -> int:
    """Number of leading results of a halo'd shard that belong to the previous rank."""
    return frame_shard(n_pairs, rank, world)[0] - frame_shard(n_pairs, rank, world, halo)[0]


def _world_rank(group=None) -> tuple[int, int]:
    """(world size, rank) of ``group``; (1, 0) when no process group exists (one process:
    ``bench.py --shard frames --gpus 1`` starts none)."""
    if not (dist.is_available() and dist.is_initialized()):
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def gather_relative_poses(T_local: torch.Tensor, status_local: torch.Tensor, n_pairs: int,
                          group=None) -> tuple[np.ndarray, np.ndarray]:
    """All-gather every rank's relative transforms (f64 [n_r,4,4]) and statuses into the
    full per-pair arrays (rank order == frame order).  Without a process group the local
    arrays are the whole sequence and are returned as they are."""
    world, _ = _world_rank(group)
    if world == 1 and not (dist.is_available() and dist.is_initialized()):
        return T_local.cpu().numpy(), status_local.cpu().numpy()
    # gloo (CPU tests, or GPU ranks sharing one card) all-gathers host tensors
    dev = torch.device("cpu") if dist.get_backend(group) == "gloo" else T_local.device
    T_local, status_local = T_local.to(dev), status_local.to(dev)
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


def run_sequence_sharded(make_frontend, L_all: torch.Tensor, R_all: torch.Tensor, stamps=None, use_ba: bool = True,
                         group=None, first_image: int = 0, n_pairs: int | None = None):
    """One sequence split over the ranks by frame pairs (the strong-scaling
    path): rank r runs the pairs frame_shard(n_pairs, r, world) on its own front end
    (``make_frontend()``), starting K-1 pairs early when local BA is on (``frame_shard(...,
    halo=K-1)``, so every owned pair's BA window spans the same K frames as on one GPU) and
    dropping those warm-up results; the relative poses and statuses are all-gathered
    (``gather_relative_poses``) and every rank composes the chain left to right in float64
    (stereo_slam.py:306, ``eval.chain``).  Returns what ``vo.run_sequence`` returns on one
    GPU for the whole sequence: (TUM rows, relative T, statuses) -- bit-identical to it.

    ``L_all[i - first_image]`` is image i: a rank may hold only the images its shard reads
    (images s-1 .. e-1 of its halo'd shard), with ``n_pairs`` the whole sequence's pair count
    (default: every image is held, n_pairs = len(L_all) - 1)."""
    from . import eval as ev
    from .vo import _check_overflow
    world, rank = _world_rank(group)
    if n_pairs is None:
        if first_image:
            raise ValueError("n_pairs is required when L_all starts past image 0")
        n_pairs = L_all.shape[0] - 1
    fe = make_frontend()
    halo = fe.ba_window - 1 if (fe.ba_window and use_ba) else 0
    s, e = frame_shard(n_pairs, rank, world, halo=halo)
    if e > s and (s - 1 < first_image or e - 1 - first_image >= L_all.shape[0]):
        raise ValueError(f"rank {rank} needs images {s - 1}..{e - 1}, holds {first_image}.."
                         f"{first_image + L_all.shape[0] - 1}")
    drop = warmup_pairs(n_pairs, rank, world, halo)
    Ts, sts = [], []
    if e > s:
        o = first_image
        fe.prime(L_all[s - 1 - o], R_all[s - 1 - o])
        for a in range(s, e, fe.B):
            b = min(a + fe.B, e)
            T, st = fe.step(L_all[a - o:b - o], R_all[a - o:b - o])
            Ts.append((T if use_ba else fe.T[:b - a]).clone())
            sts.append(st.clone())
    dev = L_all.device
    T_local = torch.cat(Ts)[drop:] if Ts else torch.zeros((0, 4, 4), dtype=torch.float64, device=dev)
    st_local = torch.cat(sts)[drop:] if sts else torch.zeros((0,), dtype=torch.int32, device=dev)
    T, S = gather_relative_poses(T_local, st_local, n_pairs, group)
    _check_overflow(S)
    valid = S != -1
    cum = ev.chain(T, valid)
    if stamps is None:
        stamps = np.arange(n_pairs + 1, dtype=np.float64)
    return ev.tum_rows(np.asarray(stamps)[1:][valid], cum), T, S


def exchange_frame_map(T_step: torch.Tensor, st_step: torch.Tensor, P3: torch.Tensor, n_points: torch.Tensor,
                       group=None, dst: int | None = None):
    """The per-step map exchange of the multi-sequence run: every rank's
    relative poses of the step (f64 [B,4,4], BA-refined with local BA), their statuses (i32 [B])
    and every frame's points3D (the back-projected, depth-filtered points PnP consumed: f32
    [B,cap,3] + i32 [B] counts, stereo_slam.py:274-289) are all-gathered (RCCL over xGMI), or,
    with ``dst`` set, gathered to that rank only (the map placed on one rank: the others send and
    receive nothing back; they get None).  Fixed shapes and device-side counts: no host
    synchronisation, the collectives queue on the current stream.  Returns (T [world,B,4,4],
    st [world,B], P3 [world,B,cap,3], n [world,B]) on the inputs' device.  Under the gloo
    backend (CPU tests, or GPU ranks sharing one card) the tensors go through host copies."""
    world = dist.get_world_size(group)
    host = dist.get_backend(group) == "gloo" and T_step.is_cuda
    dev = T_step.device
    ins = [t.contiguous().cpu() if host else t.contiguous() for t in (T_step, st_step, P3, n_points)]
    me = dist.get_rank(group)
    outs = []
    for t in ins:
        if dst is None or me == dst:
            o = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
            if dst is None:
                dist.all_gather(list(o.unbind(0)), t, group=group)
            else:
                dist.gather(t, list(o.unbind(0)), dst=dst, group=group)
            outs.append(o.to(dev) if host else o)
        else:
            dist.gather(t, None, dst=dst, group=group)
    return tuple(outs) if outs else None


def exchange_bytes(B: int, cap: int) -> int:
    """Bytes one rank contributes to a step's map exchange: T f64 [B,4,4] + status i32 [B] +
    points3D f32 [B,cap,3] + counts i32 [B] -- 1,593,856 B at 600p (B = 64, cap 2064).  The point
    sets travel at the context's capacity: a collective's shape must be known on the host when it
    is queued, and the step's point counts exist only on the device, so a compacted send would
    need a host round trip per step (the step is asynchronous by design) or a lossy fixed cap;
    ORB's retainBest keeps ties past nfeatures, so no tighter exact bound than the keypoint
    capacity exists.  DESIGN.md §6 has the measured padding share."""
    return B * (16 * 8 + 4 + cap * 3 * 4 + 4)


class GlobalMap:
    """The multi-sequence map product built from ``exchange_frame_map``'s
    output, entirely on the device: per sequence the chain of its relative poses
    (``fvo_chain_poses``: cum = cum @ T for every posed frame, stereo_slam.py:292-306) and every
    posed frame's points3D transformed by its cumulative pose and appended to one
    ``mapping.PointMap`` (``fvo_map_transform``) -- the reference's ``all_points_3D``
    (stereo_slam.py:308-318) for all ranks' sequences at once, frame-major within a rank and
    the ranks in rank order per step.  No host synchronisation: ``place`` only queues kernels
    on the current stream."""

    def __init__(self, world: int, capacity: int, device, ctx=None):
        from .mapping import PointMap
        self.world = int(world)
        self.map = PointMap(capacity, device, ctx)
        self.ctx = self.map.ctx
        self.cum = torch.eye(4, dtype=torch.float64, device=self.map.dev).repeat(self.world, 1, 1).contiguous()
        self.steps = 0

    def place(self, gathered):
        Tg, Sg, Pg, Ng = gathered
        S, n = Tg.shape[0], Tg.shape[1]
        cum, n_eff = self.ctx.chain_poses(Tg.contiguous(), Sg.contiguous(), self.cum, n_points=Ng.contiguous())
        self.map.add_frames(Pg.reshape(S * n, Pg.shape[2], Pg.shape[3]), n_eff.reshape(-1), cum.reshape(S * n, 4, 4))
        self.steps += 1

    def flush(self):
        """The map (pending kernels are on the stream ``place`` ran on: synchronise it before
        reading on the host)."""
        return self.map


class SequenceRank:
    """One rank of the sequence-per-GPU run: ``step`` = the front end's step over the rank's
    next frames, then, when the exchange is on (a process group of more than one rank, or
    ``exchange=True``), the exchange of the step's relative poses, statuses and points3D
    (``exchange_frame_map``) and, with ``map_capacity`` > 0, their placement in the
    multi-sequence map (``GlobalMap``; ``self.gmap``).  ``map_rank0_only``: the map lives on rank
    0 only -- the step data are gathered there instead of all-gathered (the other ranks send
    their ``exchange_bytes`` -- 1.59 MB per step at 600p, B = 64 -- and receive nothing), and only
    rank 0 places them.

    The exchange and the map run on their own stream behind the step's kernels: the host does
    not wait for them (nor for the step), and the next step's back stage only waits for the
    copy of this step's poses and points into the send buffers.  Returns (T, status, gathered)
    with gathered = None or the (T, st, P3, n) result, valid on ``self.stream`` (synchronise
    it, or the device, before reading it on the host).

    ``timing(True)`` brackets each step's side-stream work with HIP events (send-buffer copies,
    collectives, placement; ``exchange_stats`` reads them) and times the host call of the
    exchange (the gloo path copies through the host and blocks there)."""

    def __init__(self, frontend, group=None, map_capacity: int = 0, exchange: bool | None = None,
                 map_rank0_only: bool = False):
        self.fe = frontend
        self.group = group
        if exchange is None:
            exchange = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        self.exchange = bool(exchange)
        self.gmap = None
        self.copied = None
        self.rank0_only = bool(map_rank0_only)
        self.timed = False
        self._ev, self._host_s = [], []
        if self.exchange:
            dev, B, cap = frontend.dev, frontend.B, frontend.cap
            self.world = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
            self.stream = torch.cuda.Stream(dev)
            e = lambda shape, dt: torch.empty(shape, dtype=dt, device=dev)  # noqa: E731
            self.sT, self.sS = e((B, 4, 4), torch.float64), e((B,), torch.int32)
            self.sP, self.sN = e((B, cap, 3), torch.float32), e((B,), torch.int32)
            self.send_bytes = exchange_bytes(B, cap)
            if map_capacity > 0 and (self.rank == 0 or not self.rank0_only):
                self.gmap = GlobalMap(self.world, map_capacity, dev, ctx=frontend.ctx)

    def timing(self, on: bool):
        """Start (on) or stop recording the per-step exchange timing; starting clears it."""
        self.timed = bool(on)
        if on:
            self._ev, self._host_s = [], []

    def exchange_stats(self) -> dict | None:
        """Per-step means over the timed steps (synchronises the exchange stream): bytes this
        rank sends and receives, the side stream's time from the send copies to the end of the
        placement, the collectives' share of it, and the host time of the exchange call."""
        if not self.exchange:
            return None
        # bytes over the link: the rank's own slice of the gathered result never leaves it
        recv = self.send_bytes * (self.world - 1) if (not self.rank0_only or self.rank == 0) else 0
        # the last step's payload without the capacity padding (reads the counts: synchronises)
        self.stream.synchronize()
        useful = int(self.sN.numel()) * (16 * 8 + 4 + 4) + int(self.sN.clamp(min=0).sum().item()) * 12
        out = {"mode": ("gather to rank 0, map on rank 0 only" if self.rank0_only
                        else "all-gather, every rank places the whole map"),
               "send_bytes_per_rank_per_step": self.send_bytes, "recv_bytes_per_rank_per_step": recv,
               "useful_send_bytes_last_step": useful, "steps_timed": len(self._ev)}
        if self._ev:
            self.stream.synchronize()
            tot = [a.elapsed_time(d) for a, b, c, d in self._ev]
            col = [b.elapsed_time(c) for a, b, c, d in self._ev]
            out.update({"stream_ms_per_step": round(sum(tot) / len(tot), 4),
                        "collective_ms_per_step": round(sum(col) / len(col), 4),
                        "host_ms_per_step": round(sum(self._host_s) / len(self._host_s) * 1e3, 4)})
        return out

    def step(self, L: torch.Tensor, R: torch.Tensor):
        import time
        fe = self.fe
        dev = fe.dev
        main = torch.cuda.current_stream(dev)
        if self.copied is not None:  # the previous step's send copies read T / P3 before they are rewritten
            main.wait_event(self.copied)
        T, st = fe.step(L, R)
        if not self.exchange:
            return T, st, None
        n = L.shape[0]
        self.stream.wait_stream(main)
        with torch.cuda.stream(self.stream):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if self.timed else None
            if ev:
                ev[0].record()
            # fixed-size send buffers: frames past n are padding (status -2: not posed, 0 points)
            self.sT[:n].copy_(T)
            self.sS[:n].copy_(st)
            self.sP[:n].copy_(fe.P3[:n])
            self.sN[:n].copy_(fe.npts[:n])
            if n < fe.B:
                self.sS[n:].fill_(-2)
                self.sN[n:].zero_()
            self.copied = self.stream.record_event()
            if ev:
                ev[1].record()
            t0 = time.perf_counter()
            gathered = exchange_frame_map(self.sT, self.sS, self.sP, self.sN, self.group,
                                          dst=0 if self.rank0_only else None)
            host_s = time.perf_counter() - t0
            if ev:
                ev[2].record()
            if self.gmap is not None and gathered is not None:
                self.gmap.place(gathered)
            if ev:
                ev[3].record()
                self._ev.append(tuple(ev))
                self._host_s.append(host_s)
        return T, st, gathered


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
