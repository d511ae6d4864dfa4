"""Host-side profile of the headline wave: where does the scheduler thread spend its time?

Runs ``--warmup`` untimed waves of ``--streams`` chains (bench.py's wave mode), then one wave under cProfile, and
prints the top functions by own time and by cumulative time plus the engine's phase split.  A host function that
shows large own time inside a torch call that should be asynchronous is a hidden device sync.

    python scripts/host_profile.py --streams 1024 --warmup 2 > gpurun_out/host_profile.txt
"""
from __future__ import annotations

import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import chronos  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=1024)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--num-predict", type=int, default=64)
    ap.add_argument("--top", type=int, default=35)
    ap.add_argument("--no-cprofile", action="store_true", help="time the last wave without cProfile (for a trace)")
    a = ap.parse_args()

    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains

    eng = Engine(EngineConfig(model="llama3-8b", device="cuda", max_slots=a.streams, max_model_len=512,
                              default_num_predict=a.num_predict, seed=0))
    chains = synthetic_chains(a.streams * (a.warmup + 1), seed=1000)
    prompts = [build_prompt(c.history) for c in chains]

    def wave(batch):
        eng.blocks.clear_cache()
        reqs = [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=a.num_predict) for p in batch]
        steps = []
        while eng.has_work():
            kind = "prefill" if (eng.prefilling or eng.waiting) else "decode"
            t = time.perf_counter()
            eng.step()
            steps.append((kind, time.perf_counter() - t))
        torch.cuda.synchronize()
        return reqs, steps

    for s in range(a.warmup):
        wave(prompts[s * a.streams:(s + 1) * a.streams])
    torch.cuda.synchronize()
    for k in eng.phase_s:
        eng.phase_s[k] = 0.0
    prof = cProfile.Profile()
    t0 = time.perf_counter()
    if not a.no_cprofile:
        prof.enable()
    _, steps = wave(prompts[a.warmup * a.streams:(a.warmup + 1) * a.streams])
    prof.disable()
    wall = time.perf_counter() - t0
    print(f"wave wall {wall * 1e3:.1f} ms (under cProfile), phases "
          + json.dumps({k: round(v * 1e3, 1) for k, v in eng.phase_s.items()}) + " ms")
    print("steps (kind, host ms): " + ", ".join(f"{k[0]}{1e3 * d:.1f}" for k, d in steps))
    for key in () if a.no_cprofile else ("tottime", "cumulative"):
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats(key).print_stats(a.top)
        print(f"==== by {key} ====")
        print(buf.getvalue())


if __name__ == "__main__":
    main()
