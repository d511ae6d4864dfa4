"""CHRONOS-MI355X headline benchmark: syscall-chains/sec analyzed + p50 verdict latency, Llama-3-8B TP=1.

Metric / config from BASELINE.json.  Each rank (one per GPU, launched by torch.distributed.run for N > 1) runs an
independent Brain engine — the DP-replica deployment of SURVEY.md §2.5 — on its own share of the sensor streams:

  step = ``--streams`` kill chains arrive together (one per sensor stream); each chain's prompt is built byte-for-byte
         with the reference template (chronos_sensor.py:109-114) from synthetic fleet telemetry run through the
         in-kernel filter + chain tracker; the engine prefills them, decodes a schema-constrained JSON verdict
         (<= --num-predict tokens, the reference's ~60-token replies) for every chain, detokenizes and the verdict
         is parsed with json.loads, exactly as the sensor does (chronos_sensor.py:120).

``--mode closed`` measures the same metric in steady state instead of waves: every one of the ``--streams`` sensor
streams keeps exactly one chain in flight and submits its next chain the moment its verdict returns, so a step is
``--streams`` completed chains with no wave boundary (no straggler tail; new prompts are prefilled in the same forward
as the live decode rows — mixed steps — and the prefix cache stays warm as in a long-running server).  The headline
stays the wave form above; after it, ``--closed-steps`` closed-loop steps are timed too and reported as
``closed_loop_chains_s`` / ``closed_loop_p50_ms`` / ``closed_loop_p99_ms`` in the same JSON line.

Weights are random-init Llama-3-8B (real architecture, bf16, no checkpoint offline); data is synthetic telemetry.
Work per GPU is fixed as N grows (weak scaling).  Rank 0 prints ONE JSON line.

``--gpus N`` is authoritative: started without a launcher (no WORLD_SIZE) and N > 1, bench.py starts
``torch.distributed.run --nproc-per-node N`` on itself as a CHILD process before anything touches the GPU (never an
exec) and exits with its code; under a launcher, a WORLD_SIZE that differs from N, or N above the visible devices,
is an error — a scaling point must never silently measure fewer GPUs than it reports.
"""
from __future__ import annotations

import argparse
import collections
import json
import math
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--streams", type=int, default=1024, help="concurrent sensor streams (chains per step) per GPU")
    ap.add_argument("--num-predict", type=int, default=64)
    ap.add_argument("--single-stream", type=int, default=16, help="chains for the single-stream p50 latency")
    ap.add_argument("--burst", type=int, default=8)
    ap.add_argument("--small-burst", type=int, default=1,
                    help="decode steps per burst for a bucket of <= 2 rows (the single-stream phase; 0 = --burst)")
    ap.add_argument("--tail-burst", type=int, default=4,
                    help="decode steps per burst once a >=128-row bucket has started to drain (0 = always --burst)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-prefix-cache", action="store_true")
    ap.add_argument("--no-partial-prefix", action="store_true",
                    help="reuse only whole cached KV blocks (no copy of a partially matching block's computed slots)")
    ap.add_argument("--async-harvest", action="store_true")
    ap.add_argument("--cascade", action="store_true", help="shared-prefix cascade decode attention (off: measured "
                    "slower, profiles/r5/cascade_ab.md)")
    ap.add_argument("--kv-alloc", choices=["auto", "lazy", "full"], default="auto",
                    help="KV reservation at admission (lazy: prompt + lookahead, grown per launch, preemption; auto: "
                         "full when the pool holds every slot at max length)")
    ap.add_argument("--prefill-ramp", type=int, default=2048, help="first prefill step after idle (0 = full chunks)")
    ap.add_argument("--no-jump-forward", action="store_true", help="decode grammar-forced runs token by token")
    ap.add_argument("--jump-max-rows", type=int, default=None,
                    help="largest decode batch that parks rows for jump-forward (EngineConfig default if unset)")
    ap.add_argument("--no-mixed", action="store_true",
                    help="separate prefill steps (no prefill chunks riding in the decode batch's forward)")
    ap.add_argument("--mode", choices=["wave", "closed"], default="wave")
    ap.add_argument("--closed-steps", type=int, default=6,
                    help="wave mode: afterwards also time this many closed-loop steps (steady-state arrivals) and "
                         "report them as closed_loop_* next to the headline (0 = skip)")
    ap.add_argument("--weights", choices=["bf16", "fp8"], default="bf16",
                    help="fp8 = W8A8 e4m3 projections on the block-scaled MFMA / hipBLASLt fp8 (not the headline)")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree per replica (e.g. --model llama3-70b --tp 8): the world is split into "
                         "world/tp replicas, each a lockstep TP engine over RCCL (+ the IPC one-shot all-reduce)")
    ap.add_argument("--max-model-len", type=int, default=512)
    ap.add_argument("--sequence-parallel", action="store_true",
                    help="with --tp: Megatron sequence parallelism in prefill (reduce-scatter / all-gather)")
    return ap.parse_args()


def run_closed(a, eng, prompts, barrier, progress, steps=None, warmup=None, step_times=None):
    """Steady state: each stream resubmits on completion.  Returns (elapsed, timed requests, prefix-hit tokens);
    ``step_times`` (a list) receives the wall time of every block of --streams completions (the step-to-step spread)."""
    from chronos.sensor.prompt import VERDICT_SCHEMA

    steps = a.steps if steps is None else steps
    warmup = a.warmup if warmup is None else warmup
    done, stop = [], [False]
    # each stream's chains come from its own slice, so no prompt is ever submitted twice
    per = len(prompts) // a.streams
    pos = [0] * a.streams

    def submit(stream):
        if pos[stream] >= per:  # this stream ran out of fresh chains: it goes idle (never a repeat)
            return
        p = prompts[stream * per + pos[stream]]
        pos[stream] += 1
        eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=a.num_predict, meta={"stream": stream}, callback=on_done)

    def on_done(req):
        done.append(req)
        if not stop[0]:
            submit(req.meta["stream"])

    for s in range(a.streams):
        submit(s)
    while len(done) < warmup * a.streams and eng.has_work():
        eng.step()
    progress(f"closed-loop warmup: {len(done)} chains {dict(eng.stats)}")
    barrier()
    n0, hit0 = len(done), eng.stats["prefix_hit_tokens"]
    t0 = time.perf_counter()
    target = n0 + steps * a.streams
    mark, t_mark = n0 + a.streams, t0
    while len(done) < target and eng.has_work():
        eng.step()
        if step_times is not None and len(done) >= mark:
            now = time.perf_counter()
            step_times.append(now - t_mark)
            mark, t_mark = mark + a.streams, now
    barrier()
    elapsed = time.perf_counter() - t0
    hits = eng.stats["prefix_hit_tokens"] - hit0
    stop[0] = True
    eng.run_until_idle()  # drain the in-flight chains (untimed) before the single-stream runs
    assert len(done) >= target, "closed loop ran out of chains: generate more prompts per stream"
    return elapsed, done[n0:target], hits


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def ensure_world(a) -> int | None:
    """Reconcile --gpus with the launch.  Returns an exit code when this process only supervised a self-launch (or
    found a mismatch), None when it is a rank that should run the benchmark."""
    env_world = os.environ.get("WORLD_SIZE")
    if a.device == "cuda":
        visible = torch.cuda.device_count()  # counts devices without initialising HIP
        if a.gpus > visible:
            print(f"bench.py: --gpus {a.gpus} but only {visible} GPU(s) visible", file=sys.stderr)
            return 2
    if env_world is not None:
        if int(env_world) != a.gpus:
            print(f"bench.py: --gpus {a.gpus} disagrees with WORLD_SIZE {env_world}", file=sys.stderr)
            return 2
        return None
    if a.gpus <= 1:
        return None
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] launching {a.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def main():
    a = parse()
    rc = ensure_world(a)
    if rc is not None:
        return rc
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cuda = a.device == "cuda"
    if cuda:
        torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl" if cuda else "gloo")
    device = torch.device(f"cuda:{local}" if cuda else "cpu")
    if world % a.tp:
        raise SystemExit(f"--tp {a.tp} must divide the world size {world}")
    replica, tp_rank = rank // a.tp, rank % a.tp

    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.parallel.tp import TPContext
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains
    from chronos.utils import freeze_startup_objects

    tp = TPContext.single()
    if a.tp > 1:
        # every rank creates every replica's group (new_group is collective), keeps its own
        groups = [dist.new_group(list(range(r * a.tp, (r + 1) * a.tp))) for r in range(world // a.tp)]
        tp = TPContext(tp_rank, a.tp, groups[replica])
        if cuda:
            tp.enable_ipc_allreduce()
    cfg = EngineConfig(model=a.model, device=str(device), max_slots=a.streams, max_model_len=a.max_model_len,
                       default_num_predict=a.num_predict, decode_burst=a.burst, tail_burst=a.tail_burst,
                       small_burst=a.small_burst,
                       use_graphs=not a.no_graphs,
                       prefix_cache=not a.no_prefix_cache, partial_prefix=not a.no_partial_prefix,
                       async_harvest=a.async_harvest, seed=0,
                       prefill_ramp=a.prefill_ramp, jump_forward=not a.no_jump_forward,
                       mixed_batching=not a.no_mixed,
                       **({"jump_max_rows": a.jump_max_rows} if a.jump_max_rows is not None else {}),
                       weight_dtype=a.weights, tp_sequence_parallel=a.sequence_parallel,
                       cascade=a.cascade, kv_alloc=a.kv_alloc)
    # TP: the ranks of a replica submit the same chains in the same order and step the same deterministic scheduler,
    # so they stay in lockstep by construction (the serving path adds the leader broadcast of parallel/tp_engine.py)
    eng = Engine(cfg, tp=tp)
    freeze_startup_objects()  # no ~100 ms full-GC stalls inside the timed waves (profiles/r6/gc_pause.txt)
    total_steps = a.warmup + a.steps
    per_stream = total_steps if a.mode == "wave" else 2 * total_steps + 2  # closed loop: fast streams cycle more
    closed_warm = 2  # closed-loop warmup steps (the prefix cache and decode buckets settle)
    closed_per = 2 * (closed_warm + a.closed_steps) + 2 if a.mode == "wave" and a.closed_steps > 0 else 0
    chains = synthetic_chains(a.streams * (per_stream + closed_per) + a.single_stream, seed=1000 + replica)
    prompts = [build_prompt(c.history) for c in chains]
    n_main, n_closed = a.streams * per_stream, a.streams * closed_per

    def run_step(batch):
        # Nothing computed outside a step is reused inside it: the prefix cache starts empty every step, so only
        # chains arriving in the same wave share identical prompt-prefix KV blocks (computed once, in this step).
        eng.blocks.clear_cache()
        reqs = [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=a.num_predict) for p in batch]
        eng.run_until_idle()
        return reqs

    def barrier():
        if world > 1:
            dist.barrier()
        if cuda:
            torch.cuda.synchronize()

    def progress(msg):
        if rank == 0:
            print(f"[bench] {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)

    progress(f"engine ready: kv blocks {eng.blocks.num_blocks}, load {eng.load_seconds:.1f}s")
    if a.mode == "closed":
        elapsed, timed, hits = run_closed(a, eng, prompts[:a.streams * per_stream], barrier, progress)
    else:
        for s in range(a.warmup):
            t = time.perf_counter()
            run_step(prompts[s * a.streams:(s + 1) * a.streams])
            progress(f"warmup step {s}: {time.perf_counter() - t:.2f}s {dict(eng.stats)}")
        barrier()
        hit0 = eng.stats["prefix_hit_tokens"]
        t0 = time.perf_counter()
        timed = []
        for s in range(a.warmup, total_steps):
            ts, ph0 = time.perf_counter(), dict(eng.phase_s)
            timed += run_step(prompts[s * a.streams:(s + 1) * a.streams])
            # per-step wall time and host phase split (diagnostics; the timed region is still t0 .. the barrier below)
            dph = {k: round(v - ph0.get(k, 0.0), 3) for k, v in eng.phase_s.items()}
            progress(f"step {s} done {time.perf_counter() - ts:.3f}s {json.dumps(dph)}")
        barrier()
        elapsed = time.perf_counter() - t0
        hits = eng.stats["prefix_hit_tokens"] - hit0
        progress("phase seconds (all steps incl. warmup): "
                 + json.dumps({k: round(v, 3) for k, v in eng.phase_s.items()}))

    ok = 0
    for r in timed:
        try:
            v = json.loads(r.text)
            ok += int(isinstance(v, dict) and {"risk_score", "verdict", "reason"} <= set(v))
        except Exception:
            pass
    lat = [r.latency for r in timed]
    gen_tok = sum(len(r.out_ids) for r in timed)
    hist = collections.Counter(min(len(r.out_ids) // 4 * 4, 64) for r in timed)
    progress("verdict length histogram (4-token bins): " + json.dumps(dict(sorted(hist.items()))))
    prompt_tok = sum(len(r.prompt_ids) for r in timed)

    closed = None
    if closed_per:  # steady-state arrivals after the wave headline
        eng.blocks.clear_cache()
        c_steps: list = []
        c_el, c_timed, _ = run_closed(a, eng, prompts[n_main:n_main + n_closed], barrier, progress,
                                      steps=a.closed_steps, warmup=closed_warm, step_times=c_steps)
        closed = dict(elapsed=c_el, n=len(c_timed), lat=[r.latency for r in c_timed], steps=c_steps)
        progress(f"closed loop: {len(c_timed)} chains in {c_el:.2f}s; per-step s: "
                 + ", ".join(f"{x:.3f}" for x in c_steps))

    # single-stream latency (the reference's regime: one chain in flight)
    single = []
    for p in prompts[n_main + n_closed:]:
        single += run_step([p])
    single_lat = [r.latency for r in single[1:]] or [r.latency for r in single]
    # per-token decode time of the single stream: independent of how long the random-weight verdicts happen to be
    ss = single[1:] or single
    single_tok = [((r.t_done - r.t_first), len(r.out_ids)) for r in ss if r.t_first]

    stats = dict(elapsed=elapsed, ok=ok, n=len(timed), lat=lat, gen=gen_tok, ptok=prompt_tok, single=single_lat,
                 single_tok=single_tok, hits=hits, tp_rank=tp_rank, closed=closed)
    if world > 1:
        allst = [None] * world
        dist.all_gather_object(allst, stats)
    else:
        allst = [stats]
    if rank == 0:
        t = max(s["elapsed"] for s in allst)
        c_t = max(s["closed"]["elapsed"] for s in allst) if allst[0]["closed"] else 0.0
        allst = [s for s in allst if s["tp_rank"] == 0]  # one report per replica (its TP ranks served the same chains)
        n = sum(s["n"] for s in allst)
        oks = sum(s["ok"] for s in allst)
        lats = [x for s in allst for x in s["lat"]]
        singles = [x for s in allst for x in s["single"]]
        chains_s = n / t
        nrep = len(allst)
        metric = "syscall-chains/sec analyzed + p50 verdict latency, Llama-3-8B TP=1"
        if a.tp > 1 or a.model != "llama3-8b":
            metric = f"syscall-chains/sec analyzed + p50 verdict latency, {a.model} TP={a.tp}"
        out = {
            "metric": metric,
            "value": round(chains_s, 3),
            "unit": "chains/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * t / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if a.weights == "bf16" else "fp8-e4m3 W8A8 projections (bf16 norms/attention/KV/LM head)",
            "data": "synthetic syscall-chain telemetry (reference prompt template), random-init weights",
            "config": {
                "model": a.model, "global_batch": a.streams * nrep, "seq_len": a.max_model_len,
                "parallelism": (f"tp{a.tp}" + (f"dp{nrep}" if nrep > 1 else "")) if a.tp > 1 else
                               (f"dp{world}" if world > 1 else "tp1"),
                "streams_per_gpu": a.streams // a.tp, "streams_per_replica": a.streams, "num_predict": a.num_predict,
                "format": "verdict JSON schema (constrained decode)",
                "mode": "wave: a step = one wave of --streams chains arriving together" if a.mode == "wave" else
                        "closed: --streams streams each keep one chain in flight; a step = --streams completions",
            },
            "p50_verdict_latency_ms": round(1000 * statistics.median(lats), 2),
            "p99_verdict_latency_ms": round(1000 * sorted(lats)[max(0, math.ceil(0.99 * len(lats)) - 1)], 2),
            "single_stream_p50_latency_ms": round(1000 * statistics.median(singles), 2) if singles else None,
            "single_stream_decode_ms_per_token": round(
                1000 * sum(t for s in allst for t, _ in s["single_tok"])
                / max(1, sum(n for s in allst for _, n in s["single_tok"])), 3),
            "single_stream_verdict_tokens": round(
                sum(n for s in allst for _, n in s["single_tok"]) / max(1, sum(len(s["single_tok"]) for s in allst)), 1),
            "verdicts_valid": f"{oks}/{n}",
            "prompt_tokens_per_chain": round(sum(s["ptok"] for s in allst) / n, 1),
            "verdict_tokens_per_chain": round(sum(s["gen"] for s in allst) / n, 1),
            "generated_tokens_per_s": round(sum(s["gen"] for s in allst) / t, 1),
            "prefix_cache_hit_fraction": round(sum(s["hits"] for s in allst) / max(1, sum(s["ptok"] for s in allst)), 3),
        }
        if allst[0]["closed"]:
            c_lat = sorted(x for s in allst for x in s["closed"]["lat"])
            out.update(closed_loop_chains_s=round(sum(s["closed"]["n"] for s in allst) / c_t, 3),
                       closed_loop_p50_ms=round(1000 * statistics.median(c_lat), 2),
                       closed_loop_p99_ms=round(1000 * c_lat[max(0, math.ceil(0.99 * len(c_lat)) - 1)], 2),
                       closed_loop_steps=a.closed_steps, closed_loop_warmup=closed_warm)
            cs = allst[0]["closed"]["steps"]  # replica 0's step-to-step spread (chains/s of each --streams block)
            if cs:
                rates = [a.streams / x for x in cs]
                out.update(closed_loop_step_chains_s_min=round(min(rates), 1),
                           closed_loop_step_chains_s_max=round(max(rates), 1),
                           closed_loop_step_chains_s_cv=round(statistics.pstdev(rates) / statistics.mean(rates), 4))
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
