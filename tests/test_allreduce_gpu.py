"""IPC one-shot / two-shot all-reduce (csrc/kernels/allreduce.hip, K14) with 2 or 4 ranks sharing the box's one GPU.

Both processes map each other's exchange buffers through hipIpc handles swapped over gloo, exactly as TP ranks on
different GPUs do over xGMI.  Checks: bit-exact sums (fp32 accumulation in rank order, one bf16 rounding) over many
calls of different sizes (parity halves + device epochs), both algorithms interleaved call by call (one flag array,
monotonic values), in-place use, hipGraph capture + replay, and that the bounded spin reports (not hangs) when a peer
never arrives."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _collect(q, ps, world, timeout):
    """Results of the ranks that report within ``timeout`` s (a rank that raised reports before its peers stall in a
    collective); stragglers are killed so a hang cannot keep pytest from exiting."""
    import queue
    import time

    got, end = {}, time.monotonic() + timeout
    while len(got) < world and time.monotonic() < end:
        try:
            r, res = q.get(timeout=max(0.1, end - time.monotonic()))
            got[r] = res
        except queue.Empty:
            break
    for p in ps:
        p.join(timeout=20 if len(got) == world else 1)
        if p.is_alive():
            p.kill()
    return got


def _inputs(rank, step, n):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return (torch.randn(n, generator=g) * (rank + 1)).to(torch.bfloat16)


def _expected(world, step, n):
    acc = torch.zeros(n)
    for r in range(world):
        acc = acc + _inputs(r, step, n).float()
    return acc.to(torch.bfloat16)


def _worker(rank, world, port, q, distinct=False):
    """``distinct``: rank r on cuda:r (peer mapping over xGMI, tests/test_multi_gpu.py); else all ranks on cuda:0."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(rank if distinct else 0)
    from chronos.parallel.custom_ar import IpcAllReduce

    res = {"ok": True, "msg": ""}
    try:
        ar = IpcAllReduce(max_bytes=4 << 20, spin_limit=50_000_000)
        step = 0
        for n in (8, 4096, 8 * 1000, 1 << 20, 8, 65536, 96 * world):
            for algo in (1, 2, 0):
                if algo == 2 and n % (8 * world):
                    algo = 1
                x = _inputs(rank, step, n).cuda()
                dist.barrier()
                y = ar.all_reduce(x, out=x if step % 2 else None, algo=algo)  # alternate in-place / out-of-place
                torch.cuda.synchronize()
                if not torch.equal(y.cpu(), _expected(world, step, n)):
                    res = {"ok": False, "msg": f"mismatch n={n} algo={algo} step={step}"}
                step += 1
        ar.check()
        # graph capture: 3 all-reduces of fixed buffers (one-shot, two-shot, one-shot), replayed with new data
        n = 12288
        bufs = [torch.empty(n, dtype=torch.bfloat16, device="cuda") for _ in range(3)]
        outs = [torch.empty_like(b) for b in bufs]
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g):
                for i, (b, o) in enumerate(zip(bufs, outs)):
                    ar.all_reduce(b, out=o, algo=2 if i == 1 else 1)
        torch.cuda.synchronize()
        for rep in range(4):
            for i, b in enumerate(bufs):
                b.copy_(_inputs(rank, 500 + 3 * rep + i, n))
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            for i, o in enumerate(outs):
                if not torch.equal(o.cpu(), _expected(world, 500 + 3 * rep + i, n)):
                    res = {"ok": False, "msg": f"graph mismatch rep={rep} i={i}"}
        ar.check()
        # fused all-reduce + residual add + RMSNorm == all-reduce then ops.add_rmsnorm, bit for bit
        from chronos import ops

        for T, d in ((1, 4096), (5, 8192), (70, 1024), (3, 16384), (130, 256)):
            x = _inputs(rank, step, T * d).view(T, d).cuda()
            g = torch.Generator().manual_seed(77 + T)
            resid = torch.randn(T, d, generator=g).to(torch.bfloat16).cuda()
            w = (1 + 0.1 * torch.randn(d, generator=g)).to(torch.bfloat16).cuda()
            r_ref = resid.clone()
            y_ref = ops.add_rmsnorm(_expected(world, step, T * d).view(T, d).cuda(), r_ref, w, 1e-5)
            dist.barrier()
            y = ar.all_reduce_norm(x, resid, w, 1e-5)
            ar.all_reduce(x.view(-1).clone(), algo=1)  # interleave a plain call: shared epochs / flags
            torch.cuda.synchronize()
            if not (torch.equal(y, y_ref) and torch.equal(resid, r_ref)):
                res = {"ok": False, "msg": f"fused norm mismatch T={T} d={d}: "
                                           f"{(y.float() - y_ref.float()).abs().max().item()}"}
            step += 1
        ar.check()
        # a missing peer: only rank 0 calls; its kernel must give up and flag the error
        dist.barrier()
        if rank == 0:
            lone = IpcAllReduce.__new__(IpcAllReduce)
            lone.__dict__.update(ar.__dict__)
            lone.spin_limit = 200_000
            lone.all_reduce(_inputs(0, 0, 64).cuda())
            torch.cuda.synchronize()
            try:
                lone.check()
                res = {"ok": False, "msg": "missing peer not detected"}
            except RuntimeError:
                pass
        dist.barrier()
    except Exception as e:  # noqa: BLE001
        import traceback

        res = {"ok": False, "msg": repr(e) + "\n" + traceback.format_exc()[-3000:]}
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ipc_allreduce_ranks_share_one_gpu(world):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q), daemon=True) for r in range(world)]
    for p in ps:
        p.start()
    got = _collect(q, ps, world, 100)
    assert all(got.get(r, {}).get("ok") for r in range(world)), got


def _engine_worker(rank, world, port, q):
    """TP engine on the shared GPU: decode with the fused all-reduce + norm must produce the same tokens as the
    unfused path (the fused kernel is bit-exact), and must actually run."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.models import llama
    from chronos.parallel.tp import TPContext
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

    res = {"ok": True, "msg": ""}
    try:
        tp = TPContext.from_group()
        tp.enable_ipc_allreduce()
        tp.ipc_allreduce.spin_limit = 200_000_000
        fused_calls = [0]
        inner = tp.fast_allreduce_norm

        def counting(*a):
            y = inner(*a)
            fused_calls[0] += y is not None
            return y

        tp.fast_allreduce_norm = counting

        def gather_last(x):  # gloo has no CUDA all_gather: go through the host
            parts = [torch.empty_like(x.cpu()) for _ in range(world)]
            dist.all_gather(parts, x.contiguous().cpu())
            return torch.cat(parts, dim=-1).to(x.device)

        tp.all_gather_last = gather_last
        chains = [["[OPEN] attack_chain.sh -> /tmp/malware.bin", "[EXEC] attack_chain.sh -> curl"],
                  ["[EXEC] bash -> chmod", "[OPEN] chmod -> "]]
        outs = {}
        for fuse in (True, False):
            llama._FUSE_AR_NORM = fuse
            cfg = EngineConfig(model="tiny", device="cuda", max_slots=4, max_model_len=384, use_graphs=False,
                               decode_burst=4, seed=0)
            eng = Engine(cfg, tp=tp)
            # both ranks past their (lazy) start-up before the first IPC all-reduce spins on the peer
            dist.barrier()
            reqs = [eng.submit(build_prompt(c), fmt=VERDICT_SCHEMA, num_predict=24) for c in chains]
            eng.run_until_idle()
            outs[fuse] = [r.out_ids for r in reqs]
        tp.ipc_allreduce.check()
        if outs[True] != outs[False]:
            res = {"ok": False, "msg": f"fused {outs[True]} != unfused {outs[False]}"}
        elif fused_calls[0] == 0:
            res = {"ok": False, "msg": "fused all-reduce + norm never ran"}
    except Exception as e:  # noqa: BLE001
        import traceback

        res = {"ok": False, "msg": repr(e) + "\n" + traceback.format_exc()[-3000:]}
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_tp2_engine_fused_allreduce_norm_matches_unfused():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_engine_worker, args=(r, 2, port, q), daemon=True) for r in range(2)]
    for p in ps:
        p.start()
    got = _collect(q, ps, 2, 100)
    assert got.get(0, {}).get("ok") and got.get(1, {}).get("ok"), got
