"""Cost of a gated (skipped) decode step in the single-stream graph.

A captured burst keeps running its k steps after the last live row finished (or parked for a jump-forward run): every
kernel launches, reads the slot states and returns.  This replays the n=1 burst graph with the row already DONE and
reports the time per gated step next to a live step.

    python scripts/gated_step_cost.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains

    eng = Engine(EngineConfig(model=os.environ.get("MODEL", "llama3-8b"), device="cuda", max_slots=8,
                              max_model_len=512, seed=0, jump_forward=False))
    p = build_prompt(synthetic_chains(1, seed=7)[0].history)
    eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=64)
    eng.run_until_idle()
    (key, g), = [(k, v) for k, v in eng._graphs.items() if k[0] == 1]
    k = eng.cfg.decode_burst
    eng.s_state[0] = 0  # DONE: every step of the burst is gated
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    reps = 20
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    gated = (time.perf_counter() - t) / (reps * k)
    print(json.dumps({"graph": list(key), "burst": k, "gated_step_ms": round(1e3 * gated, 3)}))


if __name__ == "__main__":
    main()
