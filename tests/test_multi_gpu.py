"""Multi-GPU correctness harness: switches on when the box shows >= 2 GPUs, skips otherwise.

* IPC one-shot / two-shot / fused-norm all-reduce with rank r on cuda:r (peers mapped over xGMI, graph capture,
  bounded spin) — the same checks as tests/test_allreduce_gpu.py, which runs them with every rank on cuda:0;
* a TP=W engine over RCCL (+ the IPC kernels) on distinct GPUs agrees with the TP=1 engine on cuda:0;
* the DP=2 bench contract on two GPUs (``python bench.py --gpus 2`` self-launching one rank per GPU).

World sizes above the visible device count are skipped, so the 8-GPU node runs W = 2, 4, 8.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NGPU = torch.cuda.device_count()  # does not initialise HIP in the parent


def _need(world):
    if NGPU < world:
        pytest.skip(f"needs {world} GPUs, {NGPU} visible")


def _spawn(target, world, *args, timeout=240):
    import torch.multiprocessing as mp

    from test_allreduce_gpu import _collect, _port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=target, args=(r, world, port, q) + args, daemon=True) for r in range(world)]
    for p in ps:
        p.start()
    return _collect(q, ps, world, timeout)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ipc_allreduce_distinct_gpus(world):
    _need(world)
    from test_allreduce_gpu import _worker

    got = _spawn(_worker, world, True)
    assert all(got.get(r, {}).get("ok") for r in range(world)), got


CHAINS = [["[OPEN] attack_chain.sh -> /tmp/malware.bin", "[EXEC] attack_chain.sh -> curl"],
          ["[EXEC] bash -> chmod", "[OPEN] chmod -> "],
          ["[EXEC] bash -> cat", "[OPEN] cat -> /tmp/malware.bin", "[EXEC] bash -> nc"]]


def _cfg(device):
    from chronos.brain.engine.engine import EngineConfig

    return EngineConfig(model="tiny", device=device, max_slots=4, max_model_len=384, use_graphs=True,
                        decode_burst=4, seed=0)


PROMPTS = [[128000] + list(range(10, 47)), list(range(200, 219)), list(range(300, 305))]


def _first_logits(model, device):
    """fp32 logits of one 3-prompt prefill step (the first decode step's input distribution), on the host."""
    from chronos.models.llama import KVCache, make_prefill_batch

    kv = KVCache(model.cfg, model.tp, 12, 16, device)
    sb = make_prefill_batch(PROMPTS, [0, 0, 0], [[1, 2, 3], [4, 5], [6]], model.cfg, model.tp, device, max_blocks=3)
    return model.forward(sb, kv, logits_dtype=torch.float32).float().cpu().numpy()


def _tp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.cuda.set_device(rank)
    res = {"ok": True, "msg": ""}
    try:
        import torch.distributed as dist

        from chronos.parallel.tp_engine import TPEngine, init_tp
        from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

        tp, ctrl = init_tp("nccl")
        res["ipc"] = getattr(tp, "ipc_allreduce", None) is not None
        eng = TPEngine(_cfg(f"cuda:{rank}"), tp, ctrl_group=ctrl)
        res["logits"] = _first_logits(eng.engine.model, f"cuda:{rank}")  # every rank: the forward is collective
        if rank == 0:
            out = {}
            for i, c in enumerate(CHAINS):
                eng.submit(build_prompt(c), fmt=VERDICT_SCHEMA, num_predict=40,
                           callback=lambda r, i=i: out.__setitem__(i, (list(r.out_ids), r.text)))
            eng.run_until_idle()
            res["out"] = out
        else:
            eng.follower_loop()
        if res["ipc"]:
            tp.ipc_allreduce.check()
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback

        res = {"ok": False, "msg": repr(e) + "\n" + traceback.format_exc()[-3000:]}
    q.put((rank, res))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_tp_engine_distinct_gpus_matches_tp1(world):
    _need(world)
    from chronos.brain.engine.engine import Engine
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

    ref = Engine(_cfg("cuda:0"))
    ref_logits = torch.from_numpy(_first_logits(ref.model, "cuda:0"))
    reqs = [ref.submit(build_prompt(c), fmt=VERDICT_SCHEMA, num_predict=40) for c in CHAINS]
    ref.run_until_idle()
    want = [list(r.out_ids) for r in reqs]
    del ref
    torch.cuda.empty_cache()
    got = _spawn(_tp_worker, world, timeout=400)
    assert all(got.get(r, {}).get("ok") for r in range(world)), got
    assert all(got[r]["ipc"] for r in range(world)), "IPC all-reduce fell back to RCCL on a peer-capable node"
    # a systematic sharding error that still emits valid JSON fails here: bf16 logits within 2 % of max |logit|
    # (the whole-model numerics tolerance, test_model_numerics_gpu.py) and the same argmax on every prompt
    for r in range(world):
        lg = torch.from_numpy(got[r]["logits"])
        assert (lg - ref_logits).abs().max() <= 0.02 * ref_logits.abs().max(), r
        assert (lg.argmax(-1) == ref_logits.argmax(-1)).all(), r
    out = got[0]["out"]
    agree = 0.0
    for i, w in enumerate(want):
        ids, text = out[i]
        assert set(json.loads(text)) == {"risk_score", "verdict", "reason"}
        n = min(len(ids), len(w))  # different summation order across shards: greedy paths agree on a prefix
        agree += sum(a == b for a, b in zip(ids[:n], w[:n])) / max(1, n)
    assert agree / len(want) > 0.5


def test_dp2_bench_contract_on_two_gpus():
    _need(2)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--model", "tiny", "--streams", "8",
           "--steps", "1", "--warmup", "1", "--num-predict", "24", "--single-stream", "2", "--max-model-len", "384"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp2" and r["verdicts_valid"] == "16/16"


def _cp_worker(rank, world, port, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(rank)
    res = {"ok": True, "msg": ""}
    try:
        import torch.distributed as dist

        from chronos.brain.engine.engine import Engine
        from chronos.parallel.tp import TPContext
        from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

        dist.init_process_group("nccl", rank=rank, world_size=world)
        eng = Engine(_cp_cfg(f"cuda:{rank}", mode), cp=TPContext.from_group())
        req = eng.submit(build_prompt(LONG_CHAIN), fmt=VERDICT_SCHEMA, num_predict=24)
        eng.run_until_idle()
        res.update(out=list(req.out_ids), text=req.text, cp_steps=eng.stats["cp_prefill_steps"])
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback

        res = {"ok": False, "msg": repr(e) + "\n" + traceback.format_exc()[-3000:]}
    q.put((rank, res))


LONG_CHAIN = [f"[OPEN] bash -> /var/lib/app/file_{i}.dat" for i in range(40)] + ["[EXEC] bash -> curl"]


def _cp_cfg(device, mode="allgather"):
    from chronos.brain.engine.engine import EngineConfig

    return EngineConfig(model="tiny", device=device, max_slots=2, max_model_len=1024, use_graphs=True, decode_burst=4,
                        max_prefill_tokens=128, cp_min_tokens=64, prefix_cache=False, cp_mode=mode, seed=0)


@pytest.mark.parametrize("mode", ["allgather", "ulysses"])
def test_cp_prefill_distinct_gpus(mode):
    """Context-parallel long prefill over RCCL on two GPUs (both forms, SURVEY.md §2.4 C6 / §2.5 Ulysses): every
    rank decodes the verdict a single-GPU engine decodes, in lockstep."""
    _need(2)
    from chronos.brain.engine.engine import Engine
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

    ref = Engine(_cp_cfg("cuda:0"))
    r0 = ref.submit(build_prompt(LONG_CHAIN), fmt=VERDICT_SCHEMA, num_predict=24)
    ref.run_until_idle()
    want = list(r0.out_ids)
    del ref
    torch.cuda.empty_cache()
    got = _spawn(_cp_worker, 2, mode, timeout=400)
    assert all(got.get(r, {}).get("ok") for r in range(2)), got
    assert got[0]["out"] == got[1]["out"] and got[0]["cp_steps"] >= 1  # lockstep: every rank, the same verdict
    assert set(json.loads(got[0]["text"])) == {"risk_score", "verdict", "reason"}
    # the first token comes straight from the CP prefill's logits: a wrong K/V exchange changes it
    assert got[0]["out"][:1] == want[:1]
    # GEMMs over other row subsets round differently: greedy paths agree on a prefix, as in the TP test above
    n = min(len(want), len(got[0]["out"]))
    assert sum(a == b for a, b in zip(got[0]["out"][:n], want[:n])) / max(1, n) > 0.5
