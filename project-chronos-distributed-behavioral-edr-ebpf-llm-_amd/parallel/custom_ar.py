"""IPC one-shot / two-shot all-reduce for tensor-parallel decode (kernel:
csrc/kernels/allreduce.hip).

Every TP rank owns a bf16 exchange buffer (two parity halves) plus an uncached flag array; the IPC handles are
swapped once over the (gloo or RCCL) process group and every rank maps all peers' buffers.  ``all_reduce(x)`` is one
kernel launch: publish my shard, flag every peer, wait for every peer's flag, read the W shards over xGMI and sum —
one hop instead of a ring's 2(W-1), which is what decode-sized messages (16 KiB x tokens) are bound by.  The launch
takes no host-side state (the epoch lives on the device), so it is captured inside the decode hipGraph like any
other kernel.  Larger messages (prefill chunks) stay on RCCL (``TPContext.all_reduce`` picks by size).

Mid-sized messages (70B TP8 decode at large batch: 1-8 MiB) take the two-shot form: reduce-scatter of W slices
through the same exchange buffers, then an all-gather of the reduced slices.  Each rank moves 2(W-1)/W of the
message over xGMI instead of one-shot's W-1 copies, at the price of a second dependent hop.  Per link that is N
bytes (one-shot) against 2N/W (two-shot): at W = 8 two-shot wins once the saved 3N/4 outweighs one extra
flag hop (~5 us, i.e. around half a MiB at ~60 GB/s per link); at W <= 2 it saves nothing and is never picked.

A peer that never arrives makes the kernel give up after a bounded spin and set an error word (checked by
:meth:`check`), rather than hanging the GPU.

Before anything is mapped, :func:`peer_preflight` checks — collectively, so every rank reaches the same answer — that
each peer's GPU is this process's own device or one it can reach with peer access (``hipDeviceCanAccessPeer``, by
PCI bus id, so ranks that enumerate devices differently still agree).  If any rank cannot, every rank raises
:class:`PeerAccessUnavailable` and the caller (``init_tp``) logs the reason and keeps RCCL for all sizes, instead of
faulting on an unmappable buffer over xGMI.  The handle exchange is agreed the same way: one rank failing to open a
peer's buffer tears the exchange down on all ranks.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class PeerAccessUnavailable(RuntimeError):
    """The group's GPUs cannot map each other's memory; use RCCL."""


def _bus_id(index: int) -> str:
    p = torch.cuda.get_device_properties(index)
    return f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', index):02x}:" \
           f"{getattr(p, 'pci_device_id', 0):02x}"


def _probe(mine: int, peer_bus: str) -> tuple[bool, str]:
    """Can this process (on device ``mine``) map memory of the GPU with PCI id ``peer_bus``?"""
    if peer_bus == _bus_id(mine):
        return True, ""
    for j in range(torch.cuda.device_count()):
        if _bus_id(j) == peer_bus:
            if torch.cuda.can_device_access_peer(mine, j):
                return True, ""
            return False, f"no peer access from cuda:{mine} to cuda:{j} ({peer_bus})"
    return False, f"peer GPU {peer_bus} is not visible to this process"


def peer_preflight(group, device: torch.device) -> tuple[bool, str]:
    """Collective: True on every rank iff every rank can map every peer's GPU memory; else (False, first reason)."""
    world = dist.get_world_size(group)
    ids = [None] * world
    dist.all_gather_object(ids, _bus_id(device.index), group=group)
    bad = ""
    for r, bus in enumerate(ids):
        ok, why = _probe(device.index, bus)
        if not ok:
            bad = f"rank {dist.get_rank(group)} -> rank {r}: {why}"
            break
    verdicts = [None] * world
    dist.all_gather_object(verdicts, bad, group=group)
    reasons = [v for v in verdicts if v]
    return (not reasons), (reasons[0] if reasons else "")


class IpcAllReduce:
    def __init__(self, group=None, max_bytes: int = 8 << 20, device: torch.device | None = None,
                 spin_limit: int = 20_000_000, two_shot_min_bytes: int = 512 << 10):
        from .. import ops

        ops.load()
        self.C = torch.ops.chronos
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.max_bytes = max_bytes
        self.spin_limit = spin_limit
        self.two_shot_min_bytes = two_shot_min_bytes
        self.h = None
        ok, why = peer_preflight(group, self.device)
        if not ok:
            raise PeerAccessUnavailable(why)
        with torch.cuda.device(self.device):
            self.h = self.C.ar_create(self.rank, self.world, max_bytes)
        mine = self.C.ar_handles(self.h)
        allh = [None] * self.world
        dist.all_gather_object(allh, mine.numpy().tobytes(), group=group)
        table = torch.tensor([list(b) for b in allh], dtype=torch.uint8)
        err = ""
        try:
            with torch.cuda.device(self.device):
                self.C.ar_open(self.h, table)
        except RuntimeError as e:
            err = f"rank {self.rank}: {e}"
        errs = [None] * self.world
        dist.all_gather_object(errs, err, group=group)
        errs = [e for e in errs if e]
        if errs:
            self.close()
            raise PeerAccessUnavailable(f"IPC handle exchange failed ({errs[0]})")
        self.capacity = self.C.ar_capacity(self.h)  # elements per parity half

    def fits(self, x: torch.Tensor) -> bool:
        return x.dtype == torch.bfloat16 and x.is_cuda and x.numel() % 8 == 0 and x.numel() <= self.capacity

    def pick(self, x: torch.Tensor) -> int:
        """1 = one-shot, 2 = two-shot (needs numel % (8 * world) == 0)."""
        if self.world > 2 and x.numel() * x.element_size() >= self.two_shot_min_bytes \
                and x.numel() % (8 * self.world) == 0:
            return 2
        return 1

    def all_reduce(self, x: torch.Tensor, out: torch.Tensor | None = None, algo: int = 0) -> torch.Tensor:
        """Sum of ``x`` over the group (a new tensor unless ``out`` is given; may alias ``x``).  ``algo`` 0 picks by
        size (:meth:`pick`); 1 / 2 force one-shot / two-shot.  Every rank must pass the same algo for a call."""
        x = x.contiguous()
        out = torch.empty_like(x) if out is None else out
        self.C.ar_all_reduce(self.h, x, out, self.spin_limit, algo or self.pick(x))
        return out

    def all_reduce_norm(self, x: torch.Tensor, resid: torch.Tensor, w: torch.Tensor, eps: float,
                        out: torch.Tensor | None = None) -> torch.Tensor:
        """One-shot all-reduce of the [T, d] partials fused with the residual add and RMSNorm that follow a
        row-parallel projection: ``resid <- bf16(sum(x) + resid)`` in place, returns ``rmsnorm(resid) * w`` (the
        unfused all_reduce + ops.add_rmsnorm bit for bit, one launch)."""
        x = x.contiguous()
        out = torch.empty_like(x) if out is None else out
        self.C.ar_all_reduce_norm(self.h, x, resid, w, out, eps, self.spin_limit)
        return out

    def check(self) -> None:
        if self.C.ar_error(self.h):
            raise RuntimeError("IPC all-reduce: a peer did not arrive within the spin limit (rank desync?)")

    def close(self) -> None:
        if getattr(self, "h", None):
            torch.cuda.synchronize(self.device)
            self.C.ar_destroy(self.h)
            self.h = None
