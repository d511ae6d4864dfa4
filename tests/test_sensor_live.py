"""Live-source plumbing without BCC: the perf callback on kernel-padded samples, and the async live loop.

The kernel pads a PERF_SAMPLE_RAW payload so that 4 + size is a multiple of 8: a 288-byte data_t arrives as a
292-byte sample.  The callback must hand exactly one record to the tracker.  The async live loop
must keep polling while analyses are in flight (quirk Q1 on the live path).
"""
import asyncio
import ctypes
import threading
import time

import pytest

from chronos.sensor import abi
from chronos.sensor.chain import ChainTracker, NativeChainTracker
from chronos.sensor.loader import make_perf_callback
from chronos.sensor.main import live_async
from chronos.sensor.replay import attack_chain_records


def _padded_samples(records: bytes, pad: int = 4):
    """Yield (address keep-alive buffer, size) pairs as BCC's raw callback sees them."""
    for off in range(0, len(records), abi.RECORD_SIZE):
        raw = records[off: off + abi.RECORD_SIZE] + b"\xAA" * pad
        buf = ctypes.create_string_buffer(raw, len(raw))
        yield buf, len(raw)


def test_perf_callback_takes_exactly_one_record_from_padded_sample():
    got = []
    counters = {}
    cb = make_perf_callback(got.append, counters)
    recs = attack_chain_records()
    for buf, size in _padded_samples(recs):
        assert size == 292
        cb(0, ctypes.addressof(buf), size)
    assert b"".join(got) == recs
    assert counters == {"short": 0, "records": len(recs) // abi.RECORD_SIZE}
    # The records it produced feed both trackers without the "not a multiple of 288" error.
    for impl in (ChainTracker, NativeChainTracker):
        trigs = impl().feed_records(b"".join(got), kernel_filter=True)
        assert len(trigs) == 4


def test_perf_callback_counts_short_samples():
    got = []
    counters = {}
    cb = make_perf_callback(got.append, counters)
    buf = ctypes.create_string_buffer(b"x" * 100, 100)
    cb(0, ctypes.addressof(buf), 100)
    assert got == [] and counters["short"] == 1


class FakePerfSource:
    """Stands in for KernelSource: each poll() delivers one padded sample through the real perf callback."""

    def __init__(self, on_records, records: bytes):
        self.counters = {}
        self._cb = make_perf_callback(on_records, self.counters)
        self._samples = list(_padded_samples(records))
        self.polls = 0
        self.poll_times = []

    def poll(self, timeout_ms=-1):
        self.polls += 1
        self.poll_times.append(time.perf_counter())
        if not self._samples:
            raise EOFError
        buf, size = self._samples.pop(0)
        self._cb(0, ctypes.addressof(buf), size)


def test_async_live_loop_keeps_polling_while_verdicts_are_pending():
    recs = attack_chain_records()
    n_rec = len(recs) // abi.RECORD_SIZE
    srcs = []
    started = []
    release = threading.Event()

    def factory(on_records):
        s = FakePerfSource(on_records, recs)
        srcs.append(s)
        return s

    async def analyze(history):
        started.append(time.perf_counter())
        while not release.is_set():          # the Brain does not answer until every record has been polled
            await asyncio.sleep(0.01)
        return {"risk_score": 8, "verdict": "MALICIOUS", "reason": "x"}

    shown = []

    async def main():
        async def releaser():
            while srcs[0].polls <= n_rec if srcs else True:
                await asyncio.sleep(0.01)
            release.set()

        rel = asyncio.ensure_future(releaser())
        out = await live_async(factory, ChainTracker(), analyze, lambda t, r: shown.append((t.pid, r)),
                               poll_ms=1)
        await rel
        return out

    results = asyncio.run(asyncio.wait_for(main(), 30))
    src = srcs[0]
    # Every sample was polled while the first analyses were still pending (the poll thread never blocked).
    assert src.polls == n_rec + 1
    # The live path does no user-space kernel-filter pass (the BPF program filtered already), so the expected
    # triggers are those of the unfiltered records.
    n_trig = len(ChainTracker().feed_records(recs, kernel_filter=False))
    assert n_trig >= 4
    # (no analysis could finish before every sample was polled — the releaser waits for that — so a poll loop that
    # blocked on a pending verdict would have deadlocked into the wait_for timeout above)
    assert len(started) == n_trig
    assert len(results) == n_trig and len(shown) == n_trig
    assert src.counters["short"] == 0


class _FakeTable:
    def __init__(self, owner):
        self.owner = owner

    def open_perf_buffer(self, cb, page_cnt=8, lost_cb=None):
        self.owner.opened = ("perf", page_cnt)
        self.owner.cb, self.owner.lost_cb = cb, lost_cb

    def open_ring_buffer(self, cb):
        self.owner.opened = ("ringbuf", None)
        self.owner.cb = cb


class _FakeBPF:
    """Records what KernelSource asks of BCC; poll() replays queued raw samples through the opened callback."""

    last = None

    def __init__(self, src_file=None, cflags=()):
        self.src_file, self.cflags = src_file, list(cflags)
        self.attached, self.samples, self.opened = [], [], None
        _FakeBPF.last = self

    def get_syscall_fnname(self, name):
        return f"__x64_sys_{name}"

    def attach_kprobe(self, event, fn_name):
        self.attached.append((event, fn_name))

    def __getitem__(self, name):
        assert name == "events"
        return _FakeTable(self)

    def _drain(self, perf):
        while self.samples:
            buf, size = self.samples.pop(0)
            if perf:
                self.cb(3, ctypes.addressof(buf), size)
            else:
                self.cb(None, ctypes.addressof(buf), size)

    def perf_buffer_poll(self, timeout_ms=-1):
        assert self.opened[0] == "perf"
        self._drain(True)

    def ring_buffer_poll(self, timeout_ms=-1):
        assert self.opened[0] == "ringbuf"
        self._drain(False)


@pytest.mark.parametrize("transport,pad", [("perf", 4), ("ringbuf", 0)])
def test_kernel_source_wiring_with_fake_bcc(monkeypatch, transport, pad):
    """KernelSource against a stand-in `bcc` module: the BPF program file + filter include, the two kprobes on the
    arch syscall symbols (chronos_sensor.py:101-103), the transport (perf rings of page_cnt pages per CPU, or one
    ring buffer selected by -DCHRONOS_RINGBUF), and records delivered one per sample whatever the padding."""
    import sys
    import types

    from chronos.sensor import loader

    monkeypatch.setitem(sys.modules, "bcc", types.SimpleNamespace(BPF=_FakeBPF))
    got = []
    src = loader.KernelSource(got.append, page_cnt=64, strict_filter=True, transport=transport)
    b = _FakeBPF.last
    assert b.src_file == loader.BPF_SOURCE and f"-I{loader.BPF_DIR}" in b.cflags
    assert "-DCHRONOS_FILTER_STRICT" in b.cflags
    assert ("-DCHRONOS_RINGBUF=64" in b.cflags) == (transport == "ringbuf")
    assert b.attached == [("__x64_sys_execve", "syscall__execve"), ("__x64_sys_openat", "syscall__openat")]
    assert b.opened == ((transport, 64) if transport == "perf" else (transport, None))
    recs = attack_chain_records()
    b.samples = list(_padded_samples(recs, pad=pad))
    src.poll(0)
    assert b"".join(got) == recs and src.lost == 0


def test_ringbuf_pages_must_be_power_of_two():
    from chronos.sensor.loader import ringbuf_cflags

    assert ringbuf_cflags(256) == ["-DCHRONOS_RINGBUF=256"]
    with pytest.raises(ValueError):
        ringbuf_cflags(100)
