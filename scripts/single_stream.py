"""Single-sensor-stream verdict latency (BASELINE config "Llama-3 8B bf16 TP=1 on one MI355X, single sensor stream").

One chain in flight at a time, exactly like the reference's blocking analyze_sequence (chronos_sensor.py:117-119):
prefill the kill-chain prompt, decode the schema-constrained verdict, parse it.  Prints p50/p90 latency and the mean
per-token decode time; ``--ab`` runs the fused decode path (norm-in-GEMV, fused QKV+RoPE, decode gate) and the unfused
one on two engines in ONE process, interleaved (cdna_hip_programming.md §5.4 rule 24).

  python scripts/single_stream.py --chains 16 [--ab] [--out gpurun_out/single.json]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


# name -> (fused decode kernels, decode early-exit gate)
VARIANTS = {"fused": (True, True), "fused_nogate": (True, False), "unfused_gate": (False, True),
            "unfused": (False, False)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--chains", type=int, default=16)
    ap.add_argument("--num-predict", type=int, default=64)
    ap.add_argument("--burst", type=int, default=8)
    ap.add_argument("--ab", action="store_true")
    ap.add_argument("--async-harvest", action="store_true", help="harvest burst k while burst k+1 runs")
    ap.add_argument("--only", choices=list(VARIANTS), default="fused", help="variant without --ab")
    ap.add_argument("--knob-ab", default=None,
                    help="';'-separated knob sets ('name=v,name=v'), one fused engine captured under each, interleaved")
    ap.add_argument("--weights", choices=["bf16", "fp8"], default="bf16")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import torch

    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.models import llama
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains

    from chronos import ops

    ops.load()
    prompts = [build_prompt(c.history) for c in synthetic_chains(a.chains + 1, seed=7)]
    variants = list(VARIANTS) if a.ab else [a.only]
    knobsets = {}
    if a.knob_ab:
        for ks in a.knob_ab.split(";"):
            kv = dict(x.split("=") for x in ks.split(",") if x)
            knobsets[ks or "default"] = {k: int(v) for k, v in kv.items()}
        variants = list(knobsets)
    engines = {}
    for name in variants:
        fuse, gate = VARIANTS.get(name, (True, True))
        saved_split = ops._SPLIT_MAX
        for k, v in knobsets.get(name, {}).items():
            if k == "py_split_max":  # decode kv-split cap (ops.pick_nsplit), baked into the captured graph
                ops._SPLIT_MAX = v
            elif k in ("py_burst", "py_jump", "py_gemv_max_m", "py_small_burst"):  # engine decode_burst / jump_forward / GEMV routing
                pass
            else:
                torch.ops.chronos.set_knob(k, v)  # read when this engine's decode graph is captured
        llama._FUSE_NORM = fuse
        burst = knobsets.get(name, {}).get("py_burst", a.burst)
        eng = Engine(EngineConfig(model=a.model, device="cuda", max_slots=8, max_model_len=512, decode_burst=burst,
                                  small_burst=knobsets.get(name, {}).get("py_small_burst", 0),
                                  decode_gate=gate, seed=0, async_harvest=a.async_harvest, weight_dtype=a.weights,
                                  jump_forward=bool(knobsets.get(name, {}).get("py_jump", 1))))
        # capture the n=1 graph under this variant's setting
        eng.submit(prompts[0], fmt=VERDICT_SCHEMA, num_predict=a.num_predict)
        eng.run_until_idle()
        engines[name] = (eng, fuse)
        for k in knobsets.get(name, {}):
            if not k.startswith("py_"):
                torch.ops.chronos.set_knob(k, -1)  # back to the built-in default
        ops._SPLIT_MAX = saved_split
    res = {name: [] for name in variants}
    for eng, _ in engines.values():
        eng.phase_s.clear()
        eng.stats.clear()
    from chronos.ops import gemm

    gemv_m0 = gemm.GEMV_MAX_M
    for p in prompts[1:]:
        for name, (eng, fuse) in engines.items():
            llama._FUSE_NORM = fuse
            gemm.GEMV_MAX_M = knobsets.get(name, {}).get("py_gemv_max_m", gemv_m0)  # eager (jump) forwards
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=a.num_predict)
            eng.run_until_idle()
            dt = time.perf_counter() - t0
            json.loads(r.text)
            res[name].append((dt, len(r.out_ids), r.t_first - r.t_submit))
    out = {}
    for name, rows in res.items():
        lat = [x[0] for x in rows]
        toks = [x[1] for x in rows]
        ttft = [x[2] for x in rows]
        out[name] = dict(p50_ms=round(1e3 * statistics.median(lat), 2),
                         p90_ms=round(1e3 * sorted(lat)[int(0.9 * (len(lat) - 1))], 2),
                         mean_tokens=round(statistics.mean(toks), 1),
                         ttft_p50_ms=round(1e3 * statistics.median(ttft), 2),
                         ms_per_token=round(1e3 * sum(x[0] - x[2] for x in rows) / max(1, sum(toks)), 3),
                         jumps_per_chain=round(engines[name][0].stats["jumps"] / len(rows), 2),
                         jump_tokens_per_chain=round(engines[name][0].stats["jump_tokens"] / len(rows), 2),
                         jump_host_ms_per_chain=round(1e3 * engines[name][0].phase_s["jump"] / len(rows), 2),
                         bursts_per_chain=round(sum(v for k, v in engines[name][0].stats.items()
                                                    if k.startswith("bursts@")) / len(rows), 2))
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
