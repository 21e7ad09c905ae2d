"""Bag-driven runs of the reference scripts on the MI355X path.

* ``select_stereo_pairs`` — the message loop of ros_ws/src/stereo_slam.py:177-221: messages
  of both camera topics are enumerated together; a right image at ``index % frame_interval
  == 0`` forms a stereo pair with the latest left image, and consecutive selected pairs are
  matched (prev -> cur).  Poses are stamped with the right message's time (:337).
* ``run_stereo_bag`` — ingest (fvo_undistort_gray with each camera's K/dist, :184-186 /
  :196-198) + ``vo.StereoFrontEnd`` in batches + the left-to-right chain + TUM rows (the
  reference's ``est_poses_tum``; rows only for frames with >= 6 points, :292).
* ``run_mono_bag`` — mono_slam.py's loop (:88-118) over the left topic on ``vo.MonoFrontEnd``.
* ``gt_from_bag`` — gt_localisation.py:39-104: nearest-stamp GT pose per left image,
  T_rgb0_vlp16 @ [R(q) | p], TUM rows from the second image on.
"""
from __future__ import annotations

import numpy as np
import torch

from . import eval as ev
from . import rosbag, vo

LEFT, RIGHT, GT = "/dalsa_rgb/left/image_raw", "/dalsa_rgb/right/image_raw", "/gt_poses"

# stereo_slam.py:45-66
K0 = np.array([[642.9165664800531, 0., 460.1840658156501], [0., 641.9171825800378, 308.5846449100310], [0., 0., 1.]])
DIST_L = np.array([-0.060164620903866, 0.094005180631043, 0.0, 0.0, 0])
K1 = np.array([[644.4385505412966, 0., 455.1775919513420], [0., 643.5879520187435, 304.1616226347153], [0., 0., 1.]])
DIST_R = np.array([-0.057705696896734, 0.086955444511364, 0.0, 0.0, 0])
T_RGB0_RGB1 = np.array([[0.999994564612669, -0.00327143011166783, -0.000410475508767800, 0.253736175410149,
                         0.00326819763481066, 0.999965451959397, -0.00764289028177120, -0.000362553856124796,
                         0.000435464509051199, 0.00764150722461529, 0.999970708440001, -0.000621002717451192,
                         0.0, 0.0, 0.0, 1.0]])
# stereo_slam.py:270 takes np.linalg.norm(T_rgb0_rgb1[:3, 3]) of this (1, 16) array: the slice
# is the single element [0, 3], so the baseline used is 0.253736175410149.
BASELINE = float(np.linalg.norm(T_RGB0_RGB1[:3, 3]))
# gt_localisation.py:30-33
T_RGB0_VLP16 = np.array([[0.0238743541600432, -0.999707744440396, 0.00360642510766516, 0.138922870923538],
                         [-0.00736968896588375, -0.00378431903190059, -0.999965147452649, -0.177101909101325],
                         [0.999687515506770, 0.0238486947027063, -0.00745791352160211, -0.126685267545513],
                         [0.0, 0.0, 0.0, 1.0]])


def quaternion_matrix(q) -> np.ndarray:
    """tf.transformations.quaternion_matrix (xyzw) as used at gt_localisation.py:75."""
    q = np.array(q[:4], dtype=np.float64, copy=True)
    nq = np.dot(q, q)
    if nq < np.finfo(float).eps * 4.0:
        return np.identity(4)
    q *= np.sqrt(2.0 / nq)
    q = np.outer(q, q)
    return np.array(((1.0 - q[1, 1] - q[2, 2], q[0, 1] - q[2, 3], q[0, 2] + q[1, 3], 0.0),
                     (q[0, 1] + q[2, 3], 1.0 - q[0, 0] - q[2, 2], q[1, 2] - q[0, 3], 0.0),
                     (q[0, 2] - q[1, 3], q[1, 2] + q[0, 3], 1.0 - q[0, 0] - q[1, 1], 0.0),
                     (0.0, 0.0, 0.0, 1.0)), dtype=np.float64)


def select_stereo_pairs(bag: rosbag.Bag, frame_interval: int = 1, left=LEFT, right=RIGHT):
    """[(t, left Image, right Image)] of the selected stereo pairs, in the loop's order."""
    out, cur_left = [], None
    for index, (topic, msg, t) in enumerate(bag.read_messages(topics=[left, right])):
        if topic == left:
            cur_left = msg
        elif topic == right and index % frame_interval == 0 and cur_left is not None:
            out.append((t, cur_left, msg))
    return out


def _upload(msgs, dev):
    return torch.from_numpy(np.stack([rosbag.imgmsg_to_array(m) for m in msgs])).to(dev)


def run_stereo_bag(path: str, batch: int = 32, nfeatures: int = 500, frame_interval: int = 1, ba_window: int = 0,
                   device="cuda:0", K_left=K0, dist_left=DIST_L, K_right=K1, dist_right=DIST_R, baseline=BASELINE,
                   point_map=None):
    """stereo_slam.py's ORB branch over a bag -> (TUM rows f64[n,8], relative T, statuses).
    point_map: a ``mapping.PointMap`` that receives every posed frame's points3D in the map
    frame (stereo_slam.py:308-318)."""
    bag = rosbag.Bag(path)
    pairs = select_stereo_pairs(bag, frame_interval)
    if len(pairs) < 2:
        return np.zeros((0, 8)), np.zeros((0, 4, 4)), np.zeros((0,), np.int32)
    H, W = pairs[0][1].height, pairs[0][1].width
    fe = vo.StereoFrontEnd(W, H, K_left, dist_left, baseline, batch=batch, nfeatures=nfeatures, device=device,
                           ba_window=ba_window)
    ctx, dev = fe.ctx, fe.dev

    def gray(lo, hi):
        L = ctx.undistort_gray(_upload([p[1] for p in pairs[lo:hi]], dev), K_left, dist_left)
        R = ctx.undistort_gray(_upload([p[2] for p in pairs[lo:hi]], dev), K_right, dist_right)
        return L, R

    L0, R0 = gray(0, 1)
    fe.prime(L0[0], R0[0])
    Ts, sts = [], []
    cum = np.eye(4)
    for s in range(1, len(pairs), batch):
        e = min(s + batch, len(pairs))
        L, R = gray(s, e)
        T, st = fe.step(L, R)
        Ts.append(T.cpu().numpy())
        sts.append(st.cpu().numpy())
        if point_map is not None:
            cums = []
            for i in range(e - s):  # stereo_slam.py:306, frames the reference skips keep cum
                if sts[-1][i] != -1:
                    cum = np.dot(cum, Ts[-1][i])
                cums.append(cum.copy())
            keep = torch.from_numpy((sts[-1] != -1).astype(np.int32)).to(dev)
            point_map.add_frames(fe.P3[:e - s], fe.npts[:e - s] * keep, np.stack(cums))
    T = np.concatenate(Ts)
    st = np.concatenate(sts)
    valid = st != -1
    cum = ev.chain(T, valid)
    stamps = np.array([p[0].to_sec() for p in pairs[1:]])
    return ev.tum_rows(stamps[valid], cum), T, st


def run_mono_bag(path: str, batch: int = 32, nfeatures: int = 500, frame_interval: int = 1, device="cuda:0",
                 K=K0, dist=DIST_L, topic=LEFT):
    """mono_slam.py's loop (ORB + BF + findEssentialMat + recoverPose) over a bag's left topic."""
    bag = rosbag.Bag(path)
    sel = [(t, m) for index, (_, m, t) in enumerate(bag.read_messages(topics=[topic])) if index % frame_interval == 0]
    if len(sel) < 2:
        return np.zeros((0, 8)), np.zeros((0, 4, 4)), np.zeros((0,), np.int32)
    H, W = sel[0][1].height, sel[0][1].width
    fe = vo.MonoFrontEnd(W, H, K, batch=batch, nfeatures=nfeatures, device=device)
    ctx, dev = fe.ctx, fe.dev
    g0 = ctx.undistort_gray(_upload([sel[0][1]], dev), K, dist)
    fe.prime(g0[0])
    Ts, sts = [], []
    for s in range(1, len(sel), batch):
        e = min(s + batch, len(sel))
        T, st = fe.step(ctx.undistort_gray(_upload([m for _, m in sel[s:e]], dev), K, dist))
        Ts.append(T.cpu().numpy())
        sts.append(st.cpu().numpy())
    T = np.concatenate(Ts)
    st = np.concatenate(sts)
    cum = ev.chain(T, np.ones(len(T), bool))
    stamps = np.array([t.to_sec() for t, _ in sel[1:]])
    return ev.tum_rows(stamps, cum), T, st


def gt_from_bag(path: str, image_topic: str = LEFT, gt_topic: str = GT) -> np.ndarray:
    """gt_localisation.py:39-104 -> TUM rows of the ground-truth camera poses."""
    bag = rosbag.Bag(path)
    gt = {}
    for _, msg, t in bag.read_messages(topics=[gt_topic]):
        gt[t.to_sec()] = msg.pose
    stamps = np.array(list(gt.keys()))
    poses = list(gt.values())
    rows, prev = [], None
    for _, _, t in bag.read_messages(topics=[image_topic]):
        p = poses[int(np.argmin(np.abs(stamps - t.to_sec())))]
        M = quaternion_matrix([p.orientation.x, p.orientation.y, p.orientation.z, p.orientation.w])
        M[0:3, 3] = [p.position.x, p.position.y, p.position.z]
        M = np.dot(T_RGB0_VLP16, M)
        if prev is not None:
            q = ev.quaternion_from_matrix(M)
            rows.append([t.to_sec(), M[0, 3], M[1, 3], M[2, 3], q[0], q[1], q[2], q[3]])
        prev = M
    return np.array(rows, dtype=np.float64).reshape(-1, 8)
