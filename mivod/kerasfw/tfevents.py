"""Minimal TensorBoard event-file writer (no TensorFlow / tensorboard needed).

Writes ``events.out.tfevents.<time>.<host>`` TFRecord files containing
``Event{wall_time, step, summary{value{tag, simple_value}}}`` protobufs encoded
by hand, so stock TensorBoard (and Gradient's TensorBoard sync used by the
reference, /root/reference/mnist_keras.py:22-23,105) can read the scalars.
"""
from __future__ import annotations

import os
import socket
import struct
import time

_CRC_TABLE = []


def _make_table():
    poly = 0x82F63B78  # CRC-32C (Castagnoli), reflected
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        _CRC_TABLE.append(c)


def crc32c(data: bytes) -> int:
    if not _CRC_TABLE:
        _make_table()
    c = 0xFFFFFFFF
    for b in data:
        c = _CRC_TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wire: int) -> bytes:
    return _varint((num << 3) | wire)


def _len_delim(num: int, payload: bytes) -> bytes:
    return _field(num, 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int, scalars=None, file_version: str = None) -> bytes:
    ev = _field(1, 1) + struct.pack("<d", wall_time) + _field(2, 0) + _varint(int(step))
    if file_version is not None:
        ev += _len_delim(3, file_version.encode())
    if scalars:
        summ = b""
        for tag, val in scalars.items():
            v = _len_delim(1, tag.encode()) + _field(2, 5) + struct.pack("<f", float(val))
            summ += _len_delim(1, v)
        ev += _len_delim(5, summ)
    return ev


def _record(data: bytes) -> bytes:
    hdr = struct.pack("<Q", len(data))
    return hdr + struct.pack("<I", _masked_crc(hdr)) + data + struct.pack("<I", _masked_crc(data))


class EventWriter:
    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.mivod"
        self.path = os.path.join(logdir, name)
        self.f = open(self.path, "wb")
        self.f.write(_record(encode_event(time.time(), 0, file_version="brain.Event:2")))
        self.f.flush()

    def add_scalars(self, step: int, scalars: dict):
        self.f.write(_record(encode_event(time.time(), step, scalars)))

    def flush(self):
        self.f.flush()

    def close(self):
        if self.f:
            self.f.close()
            self.f = None


def read_events(path: str):
    """Decode our own event files (tests / tooling): [(step, {tag: value})]."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        i += 12
        rec = data[i:i + n]
        i += n + 4
        out.append(_parse_event(rec))
    return out


def _read_varint(b, i):
    shift = res = 0
    while True:
        x = b[i]
        i += 1
        res |= (x & 0x7F) << shift
        if not x & 0x80:
            return res, i
        shift += 7


def _parse_event(b):
    i, step, scalars = 0, 0, {}
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wire = key >> 3, key & 7
        if wire == 0:
            v, i = _read_varint(b, i)
            if num == 2:
                step = v
        elif wire == 1:
            i += 8
        elif wire == 5:
            i += 4
        elif wire == 2:
            ln, i = _read_varint(b, i)
            payload = b[i:i + ln]
            i += ln
            if num == 5:
                j = 0
                while j < len(payload):
                    k2, j = _read_varint(payload, j)
                    l2, j = _read_varint(payload, j)
                    val = payload[j:j + l2]
                    j += l2
                    tag, x, m = None, None, 0
                    while m < len(val):
                        k3, m = _read_varint(val, m)
                        if k3 >> 3 == 1:
                            l3, m = _read_varint(val, m)
                            tag = val[m:m + l3].decode()
                            m += l3
                        elif k3 >> 3 == 2:
                            (x,) = struct.unpack_from("<f", val, m)
                            m += 4
                        else:
                            break
                    if tag is not None:
                        scalars[tag] = x
    return step, scalars
