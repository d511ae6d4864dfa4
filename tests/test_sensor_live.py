"""Live-source plumbing without BCC: the perf callback on kernel-padded samples, and the async live loop.

The kernel pads a PERF_SAMPLE_RAW payload so that 4 + size is a multiple of 8: a 288-byte data_t arrives as a
292-byte sample.  The callback must hand exactly one record to the tracker.  The async live loop
must keep polling while analyses are in flight (quirk Q1 on the live path).
"""
import asyncio
import ctypes
import threading
import time

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
