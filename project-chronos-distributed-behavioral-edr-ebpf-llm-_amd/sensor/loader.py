"""Live kernel source: load ``bpf/chronos.bpf.c`` with BCC and stream raw ``data_t`` records.

Mirrors the reference start-up (chronos_sensor.py:101-103,160-163): compile the program, attach kprobes to the arch
syscall symbols of execve/openat, open the ``events`` perf buffer (64 pages per CPU by default) and poll.  Differences:
the program comes from a file that shares its filter header with the host build, records are handed over as raw
288-byte blobs (so the C++ tracker can batch them), and lost samples are counted instead of printed.

Sample size: the kernel pads a PERF_SAMPLE_RAW payload so that ``4 + size`` is a multiple of 8, so a 288-byte
``data_t`` arrives with ``size == 292``.  The reference never sees this because ``b['events'].event(data)`` casts the
pointer to the struct (chronos_sensor.py:125); here :func:`make_perf_callback` copies exactly ``RECORD_SIZE`` bytes
and counts anything shorter as a short (lost) sample.

BCC needs root, kernel headers and the ``bcc`` Python module.  None of these exist in the build container or on
the GPU box, so the BPF load is exercised only on a real sensor host; the perf callback and the poll loop around it
are unit-tested with padded fake samples (tests/test_sensor_live.py).
"""
from __future__ import annotations

import ctypes
import os
from typing import Callable

from . import abi

BPF_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bpf")
BPF_SOURCE = os.path.join(BPF_DIR, "chronos.bpf.c")


def bcc_available() -> bool:
    try:
        import bcc  # noqa: F401
    except Exception:
        return False
    return True


def make_perf_callback(on_records: Callable[[bytes], None], counters: dict) -> Callable:
    """The ``open_perf_buffer`` callback: one raw sample -> exactly one 288-byte record.

    ``data`` is the ctypes pointer BCC passes (an int address or a ``c_void_p``); ``size`` includes the kernel's
    8-byte alignment padding.  Samples shorter than a record are counted in ``counters['short']`` and dropped.
    """
    counters.setdefault("short", 0)
    counters.setdefault("records", 0)

    def _cb(cpu, data, size):
        if size < abi.RECORD_SIZE:
            counters["short"] += 1
            return
        counters["records"] += 1
        on_records(ctypes.string_at(data, abi.RECORD_SIZE))

    return _cb


def ringbuf_cflags(pages: int) -> list[str]:
    """cflags selecting the BPF ring-buffer transport (one buffer of ``pages`` 4-KiB pages, a power of two)."""
    if pages <= 0 or pages & (pages - 1):
        raise ValueError(f"ring buffer pages must be a power of two, got {pages}")
    return [f"-DCHRONOS_RINGBUF={pages}"]


class KernelSource:
    """``transport="perf"``: per-CPU perf rings of ``page_cnt`` pages (the reference).  ``transport="ringbuf"``: one
    BPF ring buffer of ``page_cnt`` pages shared by all CPUs — global event order across CPUs; a full buffer drops
    the record in the kernel (``ringbuf_output`` fails), which BCC does not report, so ``lost`` stays 0 there."""

    def __init__(self, on_records: Callable[[bytes], None], page_cnt: int = 64, strict_filter: bool = False,
                 transport: str = "perf"):
        from bcc import BPF  # noqa: WPS433 — optional dependency, imported lazily

        cflags = [f"-I{BPF_DIR}"] + (["-DCHRONOS_FILTER_STRICT"] if strict_filter else [])
        if transport == "ringbuf":
            cflags += ringbuf_cflags(page_cnt)
        elif transport != "perf":
            raise ValueError(f"transport must be perf or ringbuf, got {transport!r}")
        self.transport = transport
        self.bpf = BPF(src_file=BPF_SOURCE, cflags=cflags)
        self.bpf.attach_kprobe(event=self.bpf.get_syscall_fnname("execve"), fn_name="syscall__execve")
        self.bpf.attach_kprobe(event=self.bpf.get_syscall_fnname("openat"), fn_name="syscall__openat")
        self.counters: dict = {"lost": 0}

        def _lost(count):
            self.counters["lost"] += count

        cb = make_perf_callback(on_records, self.counters)
        if transport == "ringbuf":
            self.bpf["events"].open_ring_buffer(lambda ctx, data, size: cb(0, data, size) or 0)
        else:
            self.bpf["events"].open_perf_buffer(cb, page_cnt=page_cnt, lost_cb=_lost)

    @property
    def lost(self) -> int:
        return self.counters["lost"] + self.counters.get("short", 0)

    def poll(self, timeout_ms: int = -1) -> None:
        if self.transport == "ringbuf":
            self.bpf.ring_buffer_poll(timeout_ms)
        else:
            self.bpf.perf_buffer_poll(timeout_ms)
