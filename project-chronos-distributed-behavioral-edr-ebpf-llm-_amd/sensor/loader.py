"""Live kernel source: load ``bpf/chronos.bpf.c`` with BCC and stream raw ``data_t`` records.

Mirrors the reference start-up (chronos_sensor.py:101-103,160-163): compile the program, attach kprobes to the arch
syscall symbols of execve/openat, open the ``events`` perf buffer (64 pages per CPU by default) and poll.  Differences:
the program comes from a file that shares its filter header with the host build, records are handed over as raw
288-byte blobs (so the C++ tracker can batch them), and lost samples are counted instead of printed.

BCC needs root, kernel headers and the ``bcc`` Python module.  None of these exist in the build container or on
the GPU box, so this path is exercised only on a real sensor host; replay sources cover the same ABI in tests.
"""
from __future__ import annotations

import ctypes
import os
from typing import Callable

BPF_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bpf")
BPF_SOURCE = os.path.join(BPF_DIR, "chronos.bpf.c")


def bcc_available() -> bool:
    try:
        import bcc  # noqa: F401
    except Exception:
        return False
    return True


class KernelSource:
    def __init__(self, on_records: Callable[[bytes], None], page_cnt: int = 64, strict_filter: bool = False):
        from bcc import BPF  # noqa: WPS433 — optional dependency, imported lazily

        cflags = [f"-I{BPF_DIR}"] + (["-DCHRONOS_FILTER_STRICT"] if strict_filter else [])
        self.bpf = BPF(src_file=BPF_SOURCE, cflags=cflags)
        self.bpf.attach_kprobe(event=self.bpf.get_syscall_fnname("execve"), fn_name="syscall__execve")
        self.bpf.attach_kprobe(event=self.bpf.get_syscall_fnname("openat"), fn_name="syscall__openat")
        self.lost = 0
        self._on = on_records

        def _cb(cpu, data, size):
            self._on(ctypes.string_at(data, size))

        def _lost(count):
            self.lost += count

        self.bpf["events"].open_perf_buffer(_cb, page_cnt=page_cnt, lost_cb=_lost)

    def poll(self, timeout_ms: int = -1) -> None:
        self.bpf.perf_buffer_poll(timeout_ms)
