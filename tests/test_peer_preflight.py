"""IPC all-reduce peer-access preflight: when a rank cannot map a peer's GPU, every rank learns it
from the same collective, IpcAllReduce raises PeerAccessUnavailable everywhere, and init_tp keeps RCCL (here gloo)
for every all-reduce instead of faulting.  CPU, gloo world 2, the device probe monkeypatched."""
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


def _worker(rank, world, port, q, deny_rank):
    import torch.distributed as dist

    from chronos.parallel import custom_ar

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    custom_ar._bus_id = lambda i: f"0000:{i:02x}:00"
    custom_ar._probe = lambda mine, bus: ((False, "no peer access (probe)") if rank == deny_rank
                                         and bus != custom_ar._bus_id(mine) else (True, ""))
    torch.cuda.current_device = lambda: rank
    res = {}
    try:
        from chronos.parallel.tp_engine import init_tp

        # with every peer reachable IpcAllReduce would go on to map buffers, which needs a GPU: only the refused
        # case goes through init_tp's IPC set-up here
        tp, _ = init_tp("gloo", ipc_allreduce=deny_rank >= 0)
        ok, why = custom_ar.peer_preflight(None, torch.device("cuda", rank))
        x = torch.full((16,), float(rank + 1))
        y = tp.all_reduce(x)
        res = dict(ok=ok, why=why, fast=tp.fast_allreduce is not None, sum=y.tolist())
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        res = dict(err=repr(e))
    q.put((rank, res))


@pytest.mark.parametrize("deny_rank", [1, -1])
def test_preflight_agrees_and_falls_back(deny_rank):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, deny_rank)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(2))
    for p in ps:
        p.join(timeout=30)
    for r in range(2):
        assert "err" not in got[r], got
        assert got[r]["sum"] == [3.0] * 16 and got[r]["fast"] is False
        if deny_rank >= 0:  # both ranks see rank 1's refusal, not only rank 1
            assert got[r]["ok"] is False and "rank 1" in got[r]["why"] and "probe" in got[r]["why"]
        else:
            assert got[r]["ok"] is True and got[r]["why"] == ""
