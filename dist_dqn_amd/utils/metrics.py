"""Metrics sinks.

* `SummaryWriter` — TensorBoard event files (reference C32: chief-only
  ``tf.train.SummaryWriter`` writing the scalar ``loss`` every ``summary_freq``
  local train steps, `/root/reference/src/dqn_agent.py:37-39,131-136,255-260`).
  TF/tensorboard are not installed, so the Event/Summary protobufs and the
  TFRecord framing (length + masked CRC32C) are encoded by hand here.
* `JsonlWriter` — one JSON object per line (loss, SGD steps/s, frames/s,
  epsilon, replay size, ...).
* `EpisodeMonitor` — per-episode stats JSONL, replacing ``env.monitor``
  (reference C31, `/root/reference/src/main.py:146-148,163-164`).
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time
from typing import Dict, Optional

# ------------------------------------------------------------- CRC32C (Castagnoli)
_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def crc32c(data: bytes) -> int:
    try:
        from ..ops import _ext
        ext = _ext.load()
        if ext is not None and hasattr(ext, 'crc32c'):
            return ext.crc32c(data)
    except Exception:
        pass
    c = 0xFFFFFFFF
    for b in data:
        c = _CRC_TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ------------------------------------------------------------ protobuf encoding
def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _len_field(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_scalar_event(tag: str, value: float, step: int, wall_time: Optional[float] = None) -> bytes:
    # Summary.Value{tag=1 (string), simple_value=2 (float)}
    val = _len_field(1, tag.encode()) + _key(2, 5) + struct.pack('<f', float(value))
    summary = _len_field(1, val)                       # Summary.value = 1 (repeated)
    wt = time.time() if wall_time is None else wall_time
    # Event{wall_time=1 (double), step=2 (int64), summary=5}
    return _key(1, 1) + struct.pack('<d', wt) + _key(2, 0) + _varint(int(step)) + _len_field(5, summary)


def encode_file_version_event(wall_time: Optional[float] = None) -> bytes:
    wt = time.time() if wall_time is None else wall_time
    return _key(1, 1) + struct.pack('<d', wt) + _len_field(3, b'brain.Event:2')


def tfrecord(data: bytes) -> bytes:
    hdr = struct.pack('<Q', len(data))
    return hdr + struct.pack('<I', masked_crc(hdr)) + data + struct.pack('<I', masked_crc(data))


def read_tfrecords(path: str):
    """Yield record payloads (validates both CRCs) — used by tests."""
    with open(path, 'rb') as f:
        while True:
            hdr = f.read(8)
            if not hdr:
                return
            (n,) = struct.unpack('<Q', hdr)
            (hc,) = struct.unpack('<I', f.read(4))
            assert hc == masked_crc(hdr), 'header crc'
            data = f.read(n)
            (dc,) = struct.unpack('<I', f.read(4))
            assert dc == masked_crc(data), 'data crc'
            yield data


class SummaryWriter:
    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, 'events.out.tfevents.%d.%s' % (int(time.time()), socket.gethostname()))
        self._f = open(self.path, 'ab')
        self._f.write(tfrecord(encode_file_version_event()))
        self._f.flush()

    def add_scalar(self, tag: str, value: float, step: int):
        self._f.write(tfrecord(encode_scalar_event(tag, value, step)))
        self._f.flush()

    def add_summary(self, values: Dict[str, float], step: int):
        for k, v in values.items():
            self.add_scalar(k, v, step)

    def close(self):
        self._f.close()


class JsonlWriter:
    def __init__(self, path: str):
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        self._f = open(path, 'a')

    def write(self, **kv):
        kv.setdefault('time', time.time())
        self._f.write(json.dumps(kv) + '\n')
        self._f.flush()

    def close(self):
        self._f.close()


class EpisodeMonitor(JsonlWriter):
    def __init__(self, monitor_path: str, rank: int = 0):
        super().__init__(os.path.join(monitor_path, 'episodes.rank%d.jsonl' % rank))
        self.t0 = time.time()

    def episode(self, episode: int, length: int, reward: float):
        self.write(episode=episode, length=length, reward=reward, elapsed=time.time() - self.t0)
