"""CHRONOS sensor entry point — ``python -m chronos.sensor``.

Default behaviour equals ``sudo python3 chronos_sensor.py`` of the reference (README.md:64-69): live BCC source,
reference filters, one blocking Brain request per chain, reference console output.  Flags add the replay /
synthetic sources, the async many-in-flight client (quirk Q1), and the opt-in quirk fixes of SURVEY.md §2.8.

  --brain HOST[:PORT] | URL     Brain address (reference AI_SERVER_IP, chronos_sensor.py:9-10)
  --source bcc | attack | replay:FILE | synthetic:N
  --async N                     keep up to N chains in flight (0 = blocking, reference)
  --fixed                       enable all quirk fixes (word triggers, bounded memory, distinct ERROR, strict filter)
"""
from __future__ import annotations

import argparse
import asyncio
import sys
import threading
import time

from . import render
from .chain import ChainTracker, NativeChainTracker, TrackerConfig, Trigger
from .client import AsyncBrainClient, BrainClient, ClientConfig, brain_url, schema_format
from .replay import attack_chain_records, read_replay, synthetic_chains


def _parse(argv=None):
    ap = argparse.ArgumentParser(prog="chronos-sensor", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--brain", default="127.0.0.1:11434")
    ap.add_argument("--source", default="bcc")
    ap.add_argument("--model", default="llama3")
    ap.add_argument("--timeout", type=float, default=30.0)
    ap.add_argument("--async", dest="inflight", type=int, default=0)
    ap.add_argument("--fixed", action="store_true")
    ap.add_argument("--schema", action="store_true", help="send the verdict JSON schema as `format`")
    ap.add_argument("--python-tracker", action="store_true", help="use the pure-Python tracker (oracle)")
    ap.add_argument("--page-cnt", type=int, default=64,
                    help="perf: pages per CPU ring (reference: 64); ringbuf: pages of the one shared ring")
    ap.add_argument("--transport", choices=("perf", "ringbuf"), default="perf",
                    help="kernel -> user channel of the live source (ringbuf: global order across CPUs, kernel >= 5.8)")
    return ap.parse_args(argv)


def _url(s: str) -> str:
    if s.startswith("http"):
        return brain_url(s)
    host, _, port = s.partition(":")
    return brain_url(host, int(port) if port else 11434)


def _tracker(args):
    cfg = TrackerConfig(word_triggers=args.fixed, max_chain=64 if args.fixed else 0,
                        max_pids=65536 if args.fixed else 0)
    return ChainTracker(cfg) if args.python_tracker else NativeChainTracker(cfg)


def _records_from(source: str) -> bytes:
    if source == "attack":
        return attack_chain_records()
    if source.startswith("replay:"):
        return read_replay(source.split(":", 1)[1])
    raise ValueError(source)


def _kernel_source(on_records, args):
    from .loader import KernelSource

    return KernelSource(on_records, page_cnt=args.page_cnt, strict_filter=args.fixed, transport=args.transport)


async def live_async(src_factory, tracker, analyze, render_result, strict: bool = False,
                     poll_ms: int = 100, stop: "threading.Event | None" = None) -> list[dict]:
    """Live source with many chains in flight (quirk Q1 fix on the path where the reference actually stalls).

    The perf buffer is polled on one executor thread; records are fed to the tracker on that thread (the tracker is
    touched by no other thread), and each trigger is handed to the event loop with ``call_soon_threadsafe``, where
    ``analyze(history)`` runs as its own task.  The poll loop therefore never waits on the Brain, so the per-CPU
    rings keep draining while requests are in flight.  Ends on KeyboardInterrupt, when ``stop`` is set, or when the
    source's ``poll`` raises ``EOFError`` (replay-style fake sources); in-flight chains are awaited before return.
    """
    loop = asyncio.get_running_loop()
    tasks: set = set()
    results: list[dict] = []
    stop = stop or threading.Event()

    async def one(trig: Trigger):
        res = await analyze(trig.history)
        render_result(trig, res)
        results.append(res)

    def schedule(trig: Trigger):
        t = loop.create_task(one(trig))
        tasks.add(t)
        t.add_done_callback(tasks.discard)

    def on_records(buf: bytes):
        for trig in tracker.feed_records(buf, kernel_filter=False, strict=strict):
            loop.call_soon_threadsafe(schedule, trig)

    src = src_factory(on_records)

    def pump():
        while not stop.is_set():
            try:
                src.poll(poll_ms)
            except (KeyboardInterrupt, EOFError):
                return

    try:
        await loop.run_in_executor(None, pump)
    finally:
        stop.set()
    await asyncio.sleep(0)          # let call_soon_threadsafe callbacks queued by the last poll run
    while tasks:
        await asyncio.gather(*list(tasks))
    return results


def run(argv=None, src_factory=None) -> int:
    args = _parse(argv)
    src_factory = src_factory or (lambda on_records: _kernel_source(on_records, args))
    url = _url(args.brain)
    ccfg = ClientConfig(url=url, model=args.model, timeout=args.timeout,
                        fmt=schema_format() if args.schema else "json", retries=2 if args.fixed else 0)
    render.emit([render.banner_connect(args.brain.split(":")[0])])
    tracker = _tracker(args)
    strict = args.fixed

    if args.inflight <= 0:
        client = BrainClient(ccfg)

        def handle(trig: Trigger):
            render.emit(render.chain_lines(trig.pid, trig.history) + [render.waiting_line(trig.pid)])
            result = client.analyze(trig.history)
            render.emit(render.verdict_lines(result, distinct_errors=args.fixed))

        def on_records(buf: bytes, kernel_filter: bool):
            for trig in tracker.feed_records(buf, kernel_filter=kernel_filter, strict=strict):
                handle(trig)

        if args.source == "bcc":
            src = src_factory(lambda b: on_records(b, False))
            render.emit([render.banner_live()])
            while True:
                try:
                    src.poll()
                except (KeyboardInterrupt, EOFError):
                    return 0
        render.emit([render.banner_live()])
        if args.source.startswith("synthetic:"):
            for trig in synthetic_chains(int(args.source.split(":", 1)[1])):
                handle(trig)
        else:
            on_records(_records_from(args.source), True)
        return 0

    # Async: many chains in flight; each chain's block is printed when its verdict arrives.
    async def main_async():
        client = AsyncBrainClient(ccfg, max_inflight=args.inflight)
        if args.source == "bcc":
            render.emit([render.banner_live()])

            def show(trig: Trigger, result: dict):
                render.emit(render.chain_lines(trig.pid, trig.history) + render.verdict_lines(result, args.fixed))

            try:
                await live_async(src_factory, tracker, client.analyze, show, strict=strict)
            finally:
                await client.close()
            return
        if args.source.startswith("synthetic:"):
            trigs = synthetic_chains(int(args.source.split(":", 1)[1]))
        else:
            trigs = tracker.feed_records(_records_from(args.source), kernel_filter=True, strict=strict)
        render.emit([render.banner_live()])
        t0 = time.perf_counter()

        async def one(trig: Trigger):
            result = await client.analyze(trig.history)
            render.emit(render.chain_lines(trig.pid, trig.history) + render.verdict_lines(result, args.fixed))
            return result

        results = await asyncio.gather(*(one(t) for t in trigs))
        dt = time.perf_counter() - t0
        await client.close()
        ok = sum(1 for r in results if r.get("verdict") != "ERROR")
        print(f"[+] CHRONOS: {ok}/{len(results)} verdicts in {dt:.2f}s ({len(results) / max(dt, 1e-9):.1f} chains/s)",
              file=sys.stderr)

    asyncio.run(main_async())
    return 0


if __name__ == "__main__":
    sys.exit(run())
