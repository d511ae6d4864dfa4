"""Merge tuner outputs (scripts/tune_gemm_pp.py --out-plan / --out-table, one or more runs) into the routing plan
ops/gemm_plan.json and a readable per-shape table for profiles/.

  python scripts/apply_tune.py --plans gpurun_out/gemm_plan_small.json gpurun_out/gemm_plan_big.json \
      --tables gpurun_out/gemm_table_small.jsonl gpurun_out/gemm_table_big.jsonl --md profiles/r3_gemm_table.md

Rows of later plan files win at equal (shape, M); the table keeps every measured point (later files win too).
"""
import argparse
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plans", nargs="*", default=[])
    ap.add_argument("--tables", nargs="*", default=[])
    ap.add_argument("--out", default=os.path.join(REPO, "project-chronos-distributed-behavioral-edr-ebpf-llm-_amd",
                                                  "ops", "gemm_plan.json"))
    ap.add_argument("--md", default="")
    ap.add_argument("--jsonl", default="", help="merged table as JSON lines (for profiles/)")
    a = ap.parse_args()

    merged, qmerged, meta = {}, {}, {}
    for path in a.plans:
        with open(path) as fh:
            raw = json.load(fh)
        meta = raw.get("meta", meta)
        for dst, section in ((merged, "plans"), (qmerged, "qplans")):
            for key, rows in raw.get(section, {}).items():
                cur = {r[0]: r for r in dst.get(key, [])}
                cur.update({r[0]: r for r in rows})
                dst[key] = [cur[m] for m in sorted(cur)]
    if a.plans:
        meta = dict(meta, source="scripts/tune_gemm_pp.py on one MI355X (cold weights); merged by scripts/apply_tune.py")
        with open(a.out, "w") as fh:
            json.dump({"meta": meta, "plans": merged, "qplans": qmerged}, fh, indent=1)
        print(f"wrote {a.out}: {len(merged)} bf16 shapes, {len(qmerged)} fp8 shapes")

    recs = {}
    for path in a.tables:
        with open(path) as fh:
            for line in fh:
                if line.strip():
                    r = json.loads(line)
                    recs[(r["model"], r["op"], r["m"])] = r
    rows = sorted(recs.values(), key=lambda r: (r["model"], r["op"], r["m"]))
    if a.jsonl:
        with open(a.jsonl, "w") as fh:
            fh.writelines(json.dumps(r) + "\n" for r in rows)
    if a.md and rows:
        out = ["# Projection GEMMs: hand-written kernels vs hipBLASLt (one MI355X, cold weights)", "",
               "own = the fastest hand-written candidate: `gemv` (M <= 2), `cfg10x` = skinny config x "
               "(gemm_skinny.hip), `cfgN` = ping-pong config N (gemm_pp.hip); `_skS` = split-K S.  lib = torch.matmul "
               "(hipBLASLt) plus the separate epilogue kernel the library path needs (silu_mul / residual add).  "
               "weight TB/s = N x K x 2 bytes / time.  route = what ops/gemm_plan.json sends there (library only "
               "when it wins by > 3 %).", "",
               "| model | op | M | N | K | lib us | own us | own/lib speedup | own TF/s | own weight TB/s | own config | route |",
               "|---|---|---|---|---|---|---|---|---|---|---|---|"]
        for r in rows:
            out.append(f"| {r['model']} | {r['op']} | {r['m']} | {r['n']} | {r['k']} | {r['lib_us']} | {r['own_us']} | "
                       f"{r['speedup']} | {r['own_TF']} | {r.get('own_weight_TBs', '')} | {r['own']} | {r['route']} |")
        won = sum(r["route"] == "own" for r in rows)
        out += ["", f"hand-written kernel routed on {won}/{len(rows)} measured (shape, M) points."]
        with open(a.md, "w") as fh:
            fh.write("\n".join(out) + "\n")
        print(f"wrote {a.md}: {len(rows)} rows, own on {won}")


if __name__ == "__main__":
    main()
