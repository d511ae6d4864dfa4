"""The kernel -> user record ABI (reference chronos_sensor.py:18-23).

``struct data_t { u32 pid; char comm[16]; char argv[256]; char type[10]; }`` = 286 bytes + 2 bytes of tail padding
(4-byte alignment of the struct) = 288 bytes per perf record.  BCC exposes the fields to Python as ctypes char arrays,
which read as the bytes before the first NUL; :func:`decode` reproduces that.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

COMM_LEN = 16
PATH_LEN = 256
TYPE_LEN = 10
RECORD_SIZE = 288

EXEC = "EXEC"
OPEN = "OPEN"


class DataT(ctypes.Structure):
    _fields_ = [
        ("pid", ctypes.c_uint32),
        ("comm", ctypes.c_char * COMM_LEN),
        ("argv", ctypes.c_char * PATH_LEN),
        ("type", ctypes.c_char * TYPE_LEN),
    ]


assert ctypes.sizeof(DataT) == RECORD_SIZE, ctypes.sizeof(DataT)


@dataclass(frozen=True)
class RawEvent:
    """One decoded record; byte fields are NUL-stripped exactly as ctypes c_char arrays return them."""

    pid: int
    comm: bytes
    argv: bytes
    type: bytes


def encode(pid: int, comm: str | bytes, argv: str | bytes, etype: str | bytes) -> bytes:
    """Pack one record the way the BPF program fills it (truncating like bpf_get_current_comm / probe_read_str)."""
    d = DataT()
    d.pid = pid & 0xFFFFFFFF
    c = comm.encode() if isinstance(comm, str) else comm
    a = argv.encode() if isinstance(argv, str) else argv
    t = etype.encode() if isinstance(etype, str) else etype
    d.comm = c[: COMM_LEN - 1]
    d.argv = a[: PATH_LEN - 1]
    d.type = t[: TYPE_LEN - 1]
    return bytes(d)


def decode(buf: bytes, offset: int = 0) -> RawEvent:
    d = DataT.from_buffer_copy(buf, offset)
    return RawEvent(d.pid, d.comm, d.argv, d.type)


def iter_records(buf: bytes):
    if len(buf) % RECORD_SIZE:
        raise ValueError(f"buffer length {len(buf)} is not a multiple of {RECORD_SIZE}")
    for off in range(0, len(buf), RECORD_SIZE):
        yield decode(buf, off)
