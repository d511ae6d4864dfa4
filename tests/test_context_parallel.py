"""Context-parallel long prefill (parallel/context_parallel.py) over gloo, world 2 and 4.

Every CP rank must end the prefill with the complete KV cache of a single-rank prefill, the same last-token logits,
and the lockstep engines must return the same verdict on every rank.  Run on CPU (the reference kernels), which is
the same model code path the GPU ranks take with RCCL."""
import json
import os
import socket

import pytest
import torch


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_contiguous_pieces():
    from chronos.parallel.context_parallel import contiguous_pieces

    for n, w in [(100, 2), (1001, 4), (16, 8), (7, 4)]:
        pcs = contiguous_pieces(n, w)
        assert pcs[0][0] == 0 and pcs[-1][1] == n and all(a[1] == b[0] for a, b in zip(pcs, pcs[1:]))
        sizes = [b - a for a, b in pcs]
        assert max(sizes) - min(sizes) <= 1


def test_zigzag_pieces_balance():
    from chronos.parallel.context_parallel import rank_pieces, zigzag_pieces

    for n, w in [(100, 2), (1001, 4), (16, 8), (131072, 8)]:
        pcs = zigzag_pieces(n, w)
        assert pcs[0][0] == 0 and pcs[-1][1] == n and all(a[1] == b[0] for a, b in zip(pcs, pcs[1:]))
        sizes = [b - a for a, b in pcs]
        assert max(sizes) - min(sizes) <= 1
        mine = [p for r in range(w) for p in rank_pieces(n, w, r)]
        assert sorted(mine) == pcs  # a partition
        # causal work (sum of piece end positions) is balanced across ranks to one piece's worth
        work = [sum(b for _, b in rank_pieces(n, w, r)) for r in range(w)]
        assert max(work) - min(work) <= 2


def _cfg(**kw):
    from chronos.brain.engine.engine import EngineConfig

    base = dict(model="tiny", device="cpu", max_slots=2, max_model_len=1024, use_graphs=False, decode_burst=4,
                max_prefill_tokens=128, cp_min_tokens=64, prefix_cache=False)
    base.update(kw)
    return EngineConfig(**base)


def _long_prompt():
    from chronos.sensor.prompt import build_prompt

    hist = [f"[OPEN] bash -> /var/lib/app/file_{i}.dat" for i in range(40)] + ["[EXEC] bash -> curl"]
    return build_prompt(hist)


def _worker(rank, world, port, q, mode="allgather"):
    import torch.distributed as dist

    from chronos.brain.engine.engine import Engine
    from chronos.parallel.tp import TPContext
    from chronos.sensor.prompt import VERDICT_SCHEMA

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    eng = Engine(_cfg(cp_mode=mode), cp=TPContext.from_group())
    req = eng.submit(_long_prompt(), fmt=VERDICT_SCHEMA, num_predict=24)
    eng.run_until_idle()
    nblk = (len(req.prompt_ids) + 15) // 16
    blocks = req.blocks[:nblk] if req.blocks else None
    q.put((rank, req.out_ids, req.text, eng.stats["cp_prefill_steps"], len(req.prompt_ids),
           eng.kv.k[0][:16].float().numpy(), eng.kv.v[1][:16].float().numpy()))  # by value, not an fd
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("world,mode", [(2, "allgather"), (4, "allgather"), (2, "ulysses")])
def test_cp_engine_matches_single_rank(world, mode):
    """Both CP forms (zigzag all-gather; Ulysses head-sharded attention) end the prefill with the
    single-rank KV cache and decode the single-rank verdict."""
    import torch.multiprocessing as mp

    from chronos.brain.engine.engine import Engine
    from chronos.sensor.prompt import VERDICT_SCHEMA

    torch.manual_seed(0)
    ref = Engine(_cfg())
    r0 = ref.submit(_long_prompt(), fmt=VERDICT_SCHEMA, num_predict=24)
    ref.run_until_idle()
    assert len(r0.prompt_ids) > 2 * 128  # several CP chunks at world 2 (256 tokens per CP step)

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out_ids, text, cp_steps, plen, k0, v1 in res:
        k0, v1 = torch.from_numpy(k0), torch.from_numpy(v1)
        assert cp_steps >= 1 and plen == len(r0.prompt_ids)
        json.loads(text)
        assert out_ids == res[0][1]  # lockstep: every rank decodes the same verdict
        # the KV blocks this engine allocated hold the single-rank prefill's K/V (block ids match: same allocator)
        assert torch.allclose(k0.float(), ref.kv.k[0][:16].float(), atol=2e-2, rtol=2e-2)
        assert torch.allclose(v1.float(), ref.kv.v[1][:16].float(), atol=2e-2, rtol=2e-2)
    # greedy verdict of the CP engine equals the single-rank one at least over its first tokens (fp32 CPU GEMMs on
    # different row subsets can differ in the last bit)
    assert res[0][1][:8] == r0.out_ids[:8]


def _ulysses_gpu_worker(port, q):
    import torch.distributed as dist

    from chronos.models.llama import KVCache, build_model, make_prefill_batch
    from chronos.parallel.context_parallel import last_logits, make_ulysses_batch
    from chronos.parallel.tp import TPContext

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        model = build_model("tiny", device="cuda:0", seed=3)
        cfg = model.cfg
        g = torch.Generator().manual_seed(5)
        ids = torch.randint(0, 1000, (300,), generator=g).tolist()
        blocks = list(range(1, 1 + (40 + 300 + 15) // 16))
        out = {}
        for mode in ("plain", "ulysses"):
            kv = KVCache(cfg, TPContext.single(), 64, device="cuda:0")
            # a 40-token prefix already in the cache, then the 300-token chunk
            model.forward(make_prefill_batch([ids[:40]], [0], [blocks], cfg, TPContext.single(), "cuda:0",
                                             max_blocks=32, nqt=8), kv)
            if mode == "plain":
                lg = model.forward(make_prefill_batch([ids[40:]], [40], [blocks], cfg, TPContext.single(), "cuda:0",
                                                      max_blocks=32, nqt=8), kv)
            else:
                cp = TPContext.from_group()
                sb = make_ulysses_batch(ids[40:], 40, blocks, cfg, cp, "cuda:0", 32, nqt=8)
                lg = last_logits(model.forward(sb, kv), cp, sb.cp)
            out[mode] = (lg.float().cpu(), kv.k[1][1:8].float().cpu())
        dl = (out["plain"][0] - out["ulysses"][0]).abs().max().item()
        dk = (out["plain"][1] - out["ulysses"][1]).abs().max().item()
        q.put(("ok", dl, dk, out["plain"][0].abs().max().item()))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put(("err", repr(e) + traceback.format_exc()[-2000:], 0, 0))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_ulysses_prefill_gpu_kernels():
    """The Ulysses path on the GPU kernels (RCCL world 1: the all-to-alls are identities, the head-group K/V staging
    and the flash prefill over the staged scratch cache are real) equals a plain prefill of the same chunk."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_ulysses_gpu_worker, args=(_port(), q))
    p.start()
    st, dl, dk, mx = q.get(timeout=240)
    p.join(timeout=60)
    assert st == "ok", dl
    assert dk < 1e-2 and dl <= 0.02 * mx + 1e-2, (dk, dl, mx)
