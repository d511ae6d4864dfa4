"""Constrained sampler (csrc/kernels/sampler.hip) timing on the Llama-3 vocab: greedy over the verdict-schema automaton
for 1 row (single stream) and 1024 rows (the wave), A/B of the vectorised greedy path vs the general loop
(knob sampler_vec).   python scripts/bench_sampler.py"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from chronos import ops
    from chronos.brain.constrain import DONE, GrammarBank
    from chronos.brain.tokenizer import load_tokenizer
    from chronos.sensor.prompt import VERDICT_SCHEMA

    ops.load()
    C = torch.ops.chronos
    tok = load_tokenizer(None)
    V = 128256
    bank = GrammarBank(tok.token_bytes_list(), tok.stop_ids, V, 1024, "cuda")
    start = bank.get(VERDICT_SCHEMA).start
    out = []
    for rows in (1, 1024):
        logits = torch.randn(rows, V, device="cuda").to(torch.bfloat16)
        i32 = dict(dtype=torch.int32, device="cuda")
        res = {}
        for vec in (0, 1):
            C.set_knob("sampler_vec", vec)
            ts = []
            for _ in range(5):
                st = torch.full((rows,), start, **i32)
                rem = torch.full((rows,), 60, **i32)
                z = [torch.zeros(rows, **i32) for _ in range(4)]
                outt = torch.zeros(rows, 64, **i32)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    ops.constrained_sample(logits, None, bank.next, bank.dist, DONE, st, rem, None, None, z[0], z[1],
                                           z[2], z[3], outt)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 20 * 1e3)
            res[f"vec{vec}_us"] = round(statistics.median(ts), 1)
            res[f"vec{vec}_first_tokens"] = outt[:4, :3].tolist()
        rec = dict(rows=rows, **res)
        out.append(rec)
        print(json.dumps(rec), flush=True)
    C.set_knob("sampler_vec", 1)


if __name__ == "__main__":
    main()
