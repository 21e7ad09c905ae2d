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
  front-end step, the latest BA window's landmarks (``fvo_ba_landmarks``), the map
  exchange (``exchange_window_map``) and the multi-sequence map built from it
  (``GlobalMap``).
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


def gather_relative_poses(T_local: torch.Tensor, status_local: torch.Tensor, n_pairs: int,
                          group=None) -> tuple[np.ndarray, np.ndarray]:
    """All-gather every rank's relative transforms (f64 [n_r,4,4]) and statuses into the
    full per-pair arrays (rank order == frame order)."""
    world = dist.get_world_size(group)
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
                         group=None):
    """One sequence split over the ranks by frame pairs (the strong-scaling
    path): rank r runs the pairs frame_shard(n-1, r, world) on its own front end
    (``make_frontend()``), starting K-1 pairs early when local BA is on (``frame_shard(...,
    halo=K-1)``, so every owned pair's BA window spans the same K frames as on one GPU) and
    dropping those warm-up results; the relative poses and statuses are all-gathered
    (``gather_relative_poses``) and every rank composes the chain left to right in float64
    (stereo_slam.py:306, ``eval.chain``).  Returns what ``vo.run_sequence`` returns on one
    GPU for the whole sequence: (TUM rows, relative T, statuses) -- bit-identical to it."""
    from . import eval as ev
    from .vo import _check_overflow
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    n_pairs = L_all.shape[0] - 1
    fe = make_frontend()
    halo = fe.ba_window - 1 if (fe.ba_window and use_ba) else 0
    s, e = frame_shard(n_pairs, rank, world, halo=halo)
    drop = warmup_pairs(n_pairs, rank, world, halo)
    Ts, sts = [], []
    if e > s:
        fe.prime(L_all[s - 1], R_all[s - 1])
        for a in range(s, e, fe.B):
            b = min(a + fe.B, e)
            T, st = fe.step(L_all[a:b], R_all[a:b])
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


def exchange_window_map(T_step: torch.Tensor, st_step: torch.Tensor, lm_xyz: torch.Tensor, lm_count: torch.Tensor,
                        group=None):
    """The per-step map exchange of the multi-sequence run: every rank's
    BA-refined relative poses of the step (f64 [B,4,4]) with their statuses (i32 [B]) and its
    latest window's landmarks (f64 [Lmax,3] + i32 [1] count, fixed size) are all-gathered over
    RCCL.  Fixed shapes and device-side counts: no host synchronisation, the collectives queue
    behind the step's kernels.  Returns (T [world,B,4,4], st [world,B], xyz [world,Lmax,3],
    counts [world,1]) on the inputs' device.  Under the gloo backend (CPU tests, or GPU ranks
    sharing one card) the tensors go through host copies."""
    world = dist.get_world_size(group)
    host = dist.get_backend(group) == "gloo" and T_step.is_cuda
    dev = T_step.device
    ins = [t.contiguous().cpu() if host else t.contiguous() for t in (T_step, st_step, lm_xyz, lm_count)]
    outs = []
    for t in ins:
        o = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(o, t, group=group)
        outs.append(torch.stack(o).to(dev) if host else torch.stack(o))
    return tuple(outs)


class MapChain:
    """Host side of ``GlobalMap``: per rank the chain of the gathered relative poses, composed
    left to right in float64 exactly as ``eval.chain`` (frames with status -1 or keypoint
    overflow keep the previous pose, stereo_slam.py:292,306), and the pose that places a
    step's landmarks.  A step's last BA window ends at frame e and starts at
    s = max(0, e-K+1) (frame 0 = the primed pair); its landmarks are in camera-s
    coordinates, and the reference maps points of camera f-1 with the chain through frame f
    (pair f's points are back-projected from the previous image and transformed by the
    cumulative pose that already includes T_f, stereo_slam.py:306-310), so they are placed
    with the chain through s+1."""

    def __init__(self, world: int, window: int):
        self.world, self.K = int(world), int(window)
        self.cums = [[np.eye(4)] for _ in range(self.world)]  # cums[r][f]: rank r's chain through frame f

    def advance(self, T: np.ndarray, S: np.ndarray) -> np.ndarray:
        """T f64 [world,n,4,4], S i32 [world,n] of one step -> landmark poses f64 [world,4,4]."""
        from .vo import STATUS_KP_OVERFLOW
        land = []
        for r in range(self.world):
            ch = self.cums[r]
            for i in range(T.shape[1]):
                ok = S[r, i] != -1 and S[r, i] != STATUS_KP_OVERFLOW
                ch.append(np.dot(ch[-1], T[r, i]) if ok else ch[-1].copy())
            e = len(ch) - 1
            s = max(0, e - self.K + 1)
            land.append(ch[min(s + 1, e)])
        return np.stack(land)


class GlobalMap:
    """The multi-sequence map product built from ``exchange_window_map``'s
    output: every rank's latest-window landmarks placed in its sequence's map frame
    (``MapChain``) and appended to one ``mapping.PointMap`` -- the reference's
    ``all_points_3D`` (stereo_slam.py:306-318) for all ranks' sequences at once, one
    fvo_map_transform launch per step with the ranks' sets in rank order.

    The gathered poses reach the host through pinned buffers copied asynchronously; a step
    is placed ``lag`` steps later (its copy has long finished), so building the map never
    stalls the rank's stream.  ``flush`` places what is still queued."""

    def __init__(self, world: int, window: int, capacity: int, device, ctx=None, lag: int = 1):
        from .mapping import PointMap
        self.lag = int(lag)
        self.chain = MapChain(world, window)
        self.map = PointMap(capacity, device, ctx)
        self.counts = []  # per placed step: i32 [world] device landmark counts (test / report)
        self.queue = []

    def push(self, gathered, n: int):
        Tg, Sg, Xg, Cg = gathered
        hT = torch.empty(Tg[:, :n].shape, dtype=torch.float64, pin_memory=True)
        hS = torch.empty(Sg[:, :n].shape, dtype=torch.int32, pin_memory=True)
        hT.copy_(Tg[:, :n], non_blocking=True)
        hS.copy_(Sg[:, :n], non_blocking=True)
        X32 = Xg.to(torch.float32)  # PointCloud2 / fvo_map_transform take float32 xyz
        cnt = Cg.reshape(-1).to(torch.int32).clone()
        ev = torch.cuda.current_stream(Tg.device).record_event() if Tg.is_cuda else None
        self.queue.append((ev, hT, hS, X32, cnt, int(n)))
        while len(self.queue) > self.lag:
            self._place(self.queue.pop(0))

    def flush(self):
        while self.queue:
            self._place(self.queue.pop(0))
        return self.map

    def _place(self, item):
        ev, hT, hS, X32, cnt, n = item
        if ev is not None:
            ev.synchronize()
        land = self.chain.advance(hT.numpy(), hS.numpy())
        self.map.add_frames(X32, cnt, land)
        self.counts.append(cnt)


class SequenceRank:
    """One rank of the sequence-per-GPU run: ``step`` = the front end's step over the rank's
    next frames, then the exchange of the refined poses and of the latest BA window's
    landmarks with every other rank (``exchange_window_map``; skipped for world size 1 or
    without local BA) and, with ``map_capacity`` > 0, their placement in the multi-sequence
    map (``GlobalMap``; ``self.gmap``).  Returns (T, status, gathered) with gathered = None or
    the (T, st, xyz, counts) all-gather result."""

    def __init__(self, frontend, group=None, map_capacity: int = 0):
        self.fe = frontend
        self.group = group
        self.exchange = (dist.is_available() and dist.is_initialized() and frontend.ba_window > 0
                         and dist.get_world_size(group) > 1)
        self.gmap = None
        if self.exchange:
            dev = frontend.dev
            self.lm_out = (torch.empty((int(frontend.ctx.cfg.ba_max_landmarks), 3), dtype=torch.float64, device=dev),
                           torch.empty((1,), dtype=torch.int32, device=dev))
            if map_capacity > 0:
                self.gmap = GlobalMap(dist.get_world_size(group), frontend.ba_window, map_capacity, dev,
                                      ctx=frontend.ctx)

    def step(self, L: torch.Tensor, R: torch.Tensor):
        T, st = self.fe.step(L, R)
        gathered = None
        if self.exchange:
            xyz, cnt = self.fe.ctx.ba_landmarks(L.shape[0] - 1, out=self.lm_out)
            gathered = exchange_window_map(T, st, xyz, cnt, self.group)
            if self.gmap is not None:
                self.gmap.push(gathered, L.shape[0])
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
