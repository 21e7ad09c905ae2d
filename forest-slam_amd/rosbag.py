"""ROS bag v2.0 reader/writer and the two message types the reference reads
(SURVEY.md §8f rank 2).  Pure host code (stdlib + NumPy): no ROS installation needed.

The reference opens ``Datasets/BotanicGarden/1018_00_img10hz600p.bag`` (stereo_slam.py:35)
and iterates ``bag.read_messages(topics=['/dalsa_rgb/left/image_raw',
'/dalsa_rgb/right/image_raw'])`` (:177) and ``['/gt_poses']`` (gt_localisation.py:39),
decoding images with ``cv_bridge.imgmsg_to_cv2(msg, 'passthrough')`` (:184).  This module
restates those three pieces:

* ``Bag(path).read_messages(topics)`` -> (topic, msg, t) in timestamp order (ties: file
  order), as rosbag's index-merged iteration yields them; ``t`` is a ``Time`` with
  ``to_sec()``.  Chunks stored uncompressed or bz2 are supported (lz4 raises).
* ``Image`` (sensor_msgs/Image) and ``PoseStamped`` (geometry_msgs/PoseStamped) codecs;
  other types are returned as ``RawMessage`` (type name + bytes).
* ``imgmsg_to_array`` = ``imgmsg_to_cv2(msg, 'passthrough')`` for 8-bit encodings.
* ``BagWriter`` writes valid v2.0 bags (used by the tests and the synthetic-bag tool).

Record layout (rosbag v2.0): ``#ROSBAG V2.0\\n`` then records of
``<u32 header_len><header: u32 len + b'name=value' fields><u32 data_len><data>``; ops 0x03 bag
header, 0x05 chunk, 0x07 connection, 0x02 message data, 0x04 index data, 0x06 chunk info.
"""
from __future__ import annotations

import bz2
import io
import struct
from dataclasses import dataclass, field

import numpy as np

MAGIC = b"#ROSBAG V2.0\n"
OP_MSG, OP_BAG_HEADER, OP_INDEX, OP_CHUNK, OP_CHUNK_INFO, OP_CONNECTION = 0x02, 0x03, 0x04, 0x05, 0x06, 0x07

IMAGE_TYPE = "sensor_msgs/Image"
IMAGE_MD5 = "060021388200f6f0f447d0fcd9c64743"
POSE_TYPE = "geometry_msgs/PoseStamped"
POSE_MD5 = "d3812c3cbc69362b77dc0b19b345f8f5"


@dataclass(frozen=True, order=True)
class Time:
    secs: int
    nsecs: int

    def to_sec(self) -> float:
        return float(self.secs) + float(self.nsecs) * 1e-9

    @staticmethod
    def from_sec(t: float) -> "Time":
        s = int(np.floor(t))
        return Time(s, int(round((t - s) * 1e9)))


@dataclass
class Header:
    seq: int = 0
    stamp: Time = Time(0, 0)
    frame_id: str = ""


@dataclass
class Image:
    header: Header = field(default_factory=Header)
    height: int = 0
    width: int = 0
    encoding: str = "bgr8"
    is_bigendian: int = 0
    step: int = 0
    data: bytes = b""


@dataclass
class Point:
    x: float = 0.0
    y: float = 0.0
    z: float = 0.0


@dataclass
class Quaternion:
    x: float = 0.0
    y: float = 0.0
    z: float = 0.0
    w: float = 1.0


@dataclass
class Pose:
    position: Point = field(default_factory=Point)
    orientation: Quaternion = field(default_factory=Quaternion)


@dataclass
class PoseStamped:
    header: Header = field(default_factory=Header)
    pose: Pose = field(default_factory=Pose)


@dataclass
class RawMessage:
    type: str
    data: bytes


# ------------------------------------------------------------------ message codecs
class _R:
    def __init__(self, b: bytes):
        self.b, self.o = b, 0

    def u8(self):
        v = self.b[self.o]
        self.o += 1
        return v

    def u32(self):
        v = struct.unpack_from("<I", self.b, self.o)[0]
        self.o += 4
        return v

    def f64(self, n=1):
        v = struct.unpack_from(f"<{n}d", self.b, self.o)
        self.o += 8 * n
        return v

    def string(self) -> bytes:
        n = self.u32()
        v = self.b[self.o:self.o + n]
        self.o += n
        return bytes(v)


def _header(r: _R) -> Header:
    seq = r.u32()
    s, ns = r.u32(), r.u32()
    return Header(seq, Time(s, ns), r.string().decode())


def _enc_header(h: Header) -> bytes:
    fid = h.frame_id.encode()
    return struct.pack("<III", h.seq, h.stamp.secs, h.stamp.nsecs) + struct.pack("<I", len(fid)) + fid


def decode_image(data: bytes) -> Image:
    r = _R(data)
    h = _header(r)
    height, width = r.u32(), r.u32()
    enc = r.string().decode()
    big = r.u8()
    step = r.u32()
    return Image(h, height, width, enc, big, step, r.string())


def encode_image(m: Image) -> bytes:
    enc = m.encoding.encode()
    return (_enc_header(m.header) + struct.pack("<II", m.height, m.width) + struct.pack("<I", len(enc)) + enc +
            struct.pack("<BI", m.is_bigendian, m.step) + struct.pack("<I", len(m.data)) + bytes(m.data))


def decode_pose_stamped(data: bytes) -> PoseStamped:
    r = _R(data)
    h = _header(r)
    px, py, pz, qx, qy, qz, qw = r.f64(7)
    return PoseStamped(h, Pose(Point(px, py, pz), Quaternion(qx, qy, qz, qw)))


def encode_pose_stamped(m: PoseStamped) -> bytes:
    p, q = m.pose.position, m.pose.orientation
    return _enc_header(m.header) + struct.pack("<7d", p.x, p.y, p.z, q.x, q.y, q.z, q.w)


DECODERS = {IMAGE_TYPE: decode_image, POSE_TYPE: decode_pose_stamped}

_CHANNELS = {"mono8": 1, "8UC1": 1, "bgr8": 3, "rgb8": 3, "8UC3": 3, "bgra8": 4, "rgba8": 4, "8UC4": 4}


def imgmsg_to_array(msg: Image) -> np.ndarray:
    """cv_bridge.imgmsg_to_cv2(msg, desired_encoding='passthrough') for 8-bit encodings:
    an (H, W[, C]) uint8 view honouring the row step."""
    c = _CHANNELS.get(msg.encoding)
    if c is None:
        raise NotImplementedError(f"image encoding {msg.encoding!r} (8-bit encodings only)")
    buf = np.frombuffer(msg.data, np.uint8)
    rows = buf[:msg.height * msg.step].reshape(msg.height, msg.step)[:, :msg.width * c]
    return rows.reshape(msg.height, msg.width, c) if c > 1 else rows.reshape(msg.height, msg.width)


# ------------------------------------------------------------------ records
def _fields(hdr: bytes) -> dict:
    out, o = {}, 0
    while o < len(hdr):
        n = struct.unpack_from("<I", hdr, o)[0]
        o += 4
        kv = hdr[o:o + n]
        o += n
        k, _, v = kv.partition(b"=")
        out[k.decode()] = v
    return out


def _read_record(f):
    b = f.read(4)
    if len(b) < 4:
        return None
    hl = struct.unpack("<I", b)[0]
    hdr = f.read(hl)
    dl = struct.unpack("<I", f.read(4))[0]
    return _fields(hdr), f.read(dl)


def _u32(v: bytes) -> int:
    return struct.unpack("<I", v)[0]


def _time(v: bytes) -> Time:
    s, ns = struct.unpack("<II", v)
    return Time(s, ns)


@dataclass
class Connection:
    id: int
    topic: str
    type: str
    md5sum: str
    fields: dict


class Bag:
    """Read-only rosbag v2.0 (the subset of ``rosbag.Bag`` the reference uses)."""

    def __init__(self, path: str):
        self.path = path
        self.connections: dict[int, Connection] = {}
        self._entries = []  # (time, order, conn id, data)
        with open(path, "rb") as f:
            if f.read(len(MAGIC)) != MAGIC:
                raise ValueError(f"{path}: not a ROS bag v2.0 file")
            order = 0
            while True:
                rec = _read_record(f)
                if rec is None:
                    break
                h, data = rec
                op = h["op"][0]
                if op == OP_CHUNK:
                    comp = h.get("compression", b"none").decode()
                    if comp == "bz2":
                        data = bz2.decompress(data)
                    elif comp != "none":
                        raise NotImplementedError(f"chunk compression {comp!r} (none and bz2 are supported)")
                    cf = io.BytesIO(data)
                    while True:
                        r2 = _read_record(cf)
                        if r2 is None:
                            break
                        order = self._record(r2, order)
                else:
                    order = self._record(rec, order)
        self._entries.sort(key=lambda e: (e[0], e[1]))

    def _record(self, rec, order):
        h, data = rec
        op = h["op"][0]
        if op == OP_CONNECTION:
            cid = _u32(h["conn"])
            if cid not in self.connections:
                cf = _fields(data)
                self.connections[cid] = Connection(cid, h["topic"].decode(), cf.get("type", b"").decode(),
                                                   cf.get("md5sum", b"").decode(), cf)
        elif op == OP_MSG:
            self._entries.append((_time(h["time"]), order, _u32(h["conn"]), data))
            order += 1
        return order

    def get_message_count(self, topic_filters=None) -> int:
        ids = self._conn_ids(topic_filters)
        return sum(1 for e in self._entries if e[2] in ids)

    def _conn_ids(self, topics):
        if topics is None:
            return set(self.connections)
        if isinstance(topics, str):
            topics = [topics]
        return {c.id for c in self.connections.values() if c.topic in topics}

    def read_messages(self, topics=None, raw: bool = False):
        ids = self._conn_ids(topics)
        for t, _, cid, data in self._entries:
            if cid not in ids:
                continue
            c = self.connections[cid]
            if raw:
                yield c.topic, RawMessage(c.type, data), t
                continue
            dec = DECODERS.get(c.type)
            yield c.topic, (dec(data) if dec else RawMessage(c.type, data)), t

    def close(self):
        self._entries = []

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# ------------------------------------------------------------------ writer
def _hdr(**fields) -> bytes:
    out = b""
    for k, v in fields.items():
        kv = k.encode() + b"=" + v
        out += struct.pack("<I", len(kv)) + kv
    return out


def _rec(header: bytes, data: bytes) -> bytes:
    return struct.pack("<I", len(header)) + header + struct.pack("<I", len(data)) + data


def _conn_rec(cid: int, topic: str, typ: str, md5: str) -> bytes:
    data = _hdr(topic=topic.encode(), type=typ.encode(), md5sum=md5.encode(), message_definition=b"")
    return _rec(_hdr(op=bytes([OP_CONNECTION]), conn=struct.pack("<I", cid), topic=topic.encode()), data)


class BagWriter:
    """Minimal rosbag v2.0 writer: one uncompressed (or bz2) chunk per ``chunk_msgs`` messages,
    per-chunk index records, connection + chunk-info records at the end."""

    def __init__(self, path: str, chunk_msgs: int = 64, compression: str = "none"):
        if compression not in ("none", "bz2"):
            raise ValueError("compression must be 'none' or 'bz2'")
        self.f = open(path, "wb")
        self.f.write(MAGIC)
        self._hdr_pos = self.f.tell()
        self.f.write(b"\0" * 4096)  # bag header placeholder (rewritten on close)
        self.chunk_msgs, self.compression = chunk_msgs, compression
        self.conns: dict[str, tuple[int, str, str]] = {}
        self._pending = []
        self._chunk_infos = []

    def _conn(self, topic, typ, md5):
        if topic not in self.conns:
            self.conns[topic] = (len(self.conns), typ, md5)
        return self.conns[topic][0]

    def write(self, topic: str, msg, t: Time | float):
        if isinstance(t, (int, float)):
            t = Time.from_sec(float(t))
        if isinstance(msg, Image):
            cid, data = self._conn(topic, IMAGE_TYPE, IMAGE_MD5), encode_image(msg)
        elif isinstance(msg, PoseStamped):
            cid, data = self._conn(topic, POSE_TYPE, POSE_MD5), encode_pose_stamped(msg)
        else:
            raise TypeError("BagWriter writes Image and PoseStamped messages")
        self._pending.append((cid, t, data))
        if len(self._pending) >= self.chunk_msgs:
            self._flush()

    def _flush(self):
        if not self._pending:
            return
        body = io.BytesIO()
        seen = set()
        offsets = {}
        for cid, t, data in self._pending:
            if cid not in seen:
                topic = next(k for k, v in self.conns.items() if v[0] == cid)
                _, typ, md5 = self.conns[topic]
                body.write(_conn_rec(cid, topic, typ, md5))
                seen.add(cid)
            offsets.setdefault(cid, []).append((t, body.tell()))
            body.write(_rec(_hdr(op=bytes([OP_MSG]), conn=struct.pack("<I", cid),
                                 time=struct.pack("<II", t.secs, t.nsecs)), data))
        raw = body.getvalue()
        payload = bz2.compress(raw) if self.compression == "bz2" else raw
        pos = self.f.tell()
        self.f.write(_rec(_hdr(op=bytes([OP_CHUNK]), compression=self.compression.encode(),
                               size=struct.pack("<I", len(raw))), payload))
        times = [t for _, t, _ in self._pending]
        for cid, lst in offsets.items():
            idx = b"".join(struct.pack("<III", t.secs, t.nsecs, o) for t, o in lst)
            self.f.write(_rec(_hdr(op=bytes([OP_INDEX]), ver=struct.pack("<I", 1), conn=struct.pack("<I", cid),
                                   count=struct.pack("<I", len(lst))), idx))
        self._chunk_infos.append((pos, min(times), max(times), {c: len(v) for c, v in offsets.items()}))
        self._pending = []

    def close(self):
        self._flush()
        index_pos = self.f.tell()
        for topic, (cid, typ, md5) in self.conns.items():
            self.f.write(_conn_rec(cid, topic, typ, md5))
        for pos, t0, t1, counts in self._chunk_infos:
            data = b"".join(struct.pack("<II", c, n) for c, n in counts.items())
            self.f.write(_rec(_hdr(op=bytes([OP_CHUNK_INFO]), ver=struct.pack("<I", 1), chunk_pos=struct.pack("<Q", pos),
                                   start_time=struct.pack("<II", t0.secs, t0.nsecs),
                                   end_time=struct.pack("<II", t1.secs, t1.nsecs),
                                   count=struct.pack("<I", len(counts))), data))
        hdr = _hdr(op=bytes([OP_BAG_HEADER]), index_pos=struct.pack("<Q", index_pos),
                   conn_count=struct.pack("<I", len(self.conns)), chunk_count=struct.pack("<I", len(self._chunk_infos)))
        pad = 4096 - 4 - len(hdr) - 4
        self.f.seek(self._hdr_pos)
        self.f.write(_rec(hdr, b" " * pad))
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def image_message(arr: np.ndarray, stamp: Time, encoding: str = "bgr8", seq: int = 0, frame_id: str = "") -> Image:
    arr = np.ascontiguousarray(arr, np.uint8)
    h, w = arr.shape[:2]
    c = 1 if arr.ndim == 2 else arr.shape[2]
    return Image(Header(seq, stamp, frame_id), h, w, encoding, 0, w * c, arr.tobytes())
