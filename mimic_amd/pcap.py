"""Captured-pcap ingest for host-resident batches (BASELINE.json north_star: "captured pcap / ctx
JSON / NIC buffers").  Classic libpcap files (micro- or nanosecond timestamps, either byte
order, LINKTYPE_ETHERNET) are read into the batch layout mimic_run_xdp_host / XDPBatch take:
one contiguous byte buffer with each frame at an aligned offset, preceded by `headroom` and
followed by `tailroom` bytes (context_xdp_md.go:47-115 lays out packet memory the same way).
pcapng is not read.
"""
from __future__ import annotations

import struct
from typing import Iterable, Tuple

import numpy as np

LINKTYPE_ETHERNET = 1
_MAGIC = {b"\xd4\xc3\xb2\xa1": ("<", 1000), b"\xa1\xb2\xc3\xd4": (">", 1000),
          b"\x4d\x3c\xb2\xa1": ("<", 1), b"\xa1\xb2\x3c\x4d": (">", 1)}


def read_pcap(path_or_bytes, headroom: int = 0, tailroom: int = 0, align: int = 64, max_packets: int = 0):
    """-> (buf uint8, off uint64, lens uint32, ts_ns uint64, linktype).  Frames keep their captured
    bytes (incl_len); snap-truncated frames are passed as captured."""
    data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray, memoryview)) else open(path_or_bytes, "rb").read()
    data = memoryview(bytes(data))
    if len(data) < 24 or bytes(data[:4]) not in _MAGIC:
        raise ValueError("not a classic pcap file")
    end, tick = _MAGIC[bytes(data[:4])]
    _, _, _, _, _, linktype = struct.unpack_from(end + "HHiIII", data, 4)
    recs = []
    p = 24
    while p + 16 <= len(data):
        sec, frac, incl, _orig = struct.unpack_from(end + "IIII", data, p)
        p += 16
        if p + incl > len(data):
            raise ValueError("truncated pcap record")
        recs.append((p, incl, sec * 1_000_000_000 + frac * tick))
        p += incl
        if max_packets and len(recs) >= max_packets:
            break
    n = len(recs)
    lens = np.array([r[1] for r in recs], dtype=np.uint32)
    span = (lens.astype(np.uint64) + headroom + tailroom + align - 1) // align * align
    off = np.zeros(n, dtype=np.uint64)
    if n:
        off[1:] = np.cumsum(span[:-1])
    total = int(off[-1] + span[-1]) if n else 0
    buf = np.zeros(max(total, 1), dtype=np.uint8)
    raw = np.frombuffer(data, dtype=np.uint8)
    for i, (q, incl, _) in enumerate(recs):
        o = int(off[i]) + headroom
        buf[o:o + incl] = raw[q:q + incl]
    ts = np.array([r[2] for r in recs], dtype=np.uint64)
    return buf, off, lens, ts, linktype


def write_pcap(frames: Iterable[bytes], ts_ns: Iterable[int] = (), nanos: bool = False, snaplen: int = 65535,
               linktype: int = LINKTYPE_ETHERNET) -> bytes:
    """A classic little-endian pcap file of `frames` (for fixtures and round trips)."""
    frames = list(frames)
    ts = list(ts_ns) or [i * 1000 for i in range(len(frames))]
    out = bytearray(struct.pack("<IHHiIII", 0xA1B23C4D if nanos else 0xA1B2C3D4, 2, 4, 0, 0, snaplen, linktype))
    for f, t in zip(frames, ts):
        frac = t % 1_000_000_000 if nanos else (t % 1_000_000_000) // 1000
        out += struct.pack("<IIII", t // 1_000_000_000, frac, len(f), len(f)) + bytes(f)
    return bytes(out)


def batch_to_frames(buf, off, lens, headroom: int = 0) -> Tuple[bytes, ...]:
    return tuple(bytes(buf[int(o) + headroom:int(o) + headroom + int(n)]) for o, n in zip(off, lens))
