"""Tensor-parallel context: the collectives the Llama forward needs.

One process per GPU.  ``torch.distributed`` with backend ``"nccl"`` is RCCL on ROCm and runs over xGMI between the
GPUs of a node; ``"gloo"`` serves the CPU tests.  Column-parallel wqkv / w_gu, row-parallel wo / w_down, vocab-parallel
embedding and LM head, so a layer needs exactly two all-reduces (after o_proj and after down_proj).

The small decode-time all-reduces (70B TP8: 160 per step at 16 KiB x batch) are latency-bound; ``allreduce`` lets a
faster one-shot implementation (parallel/custom_ar.py) take messages under its size cap, RCCL takes the rest.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.distributed as dist


@dataclass
class TPContext:
    rank: int = 0
    world: int = 1
    group: Optional[object] = None
    fast_allreduce: Optional[Callable[[torch.Tensor], Optional[torch.Tensor]]] = None
    # (x, resid, w, eps) -> normalised rows, or None when the fused IPC kernel cannot take the message
    fast_allreduce_norm: Optional[Callable[..., Optional[torch.Tensor]]] = None

    @classmethod
    def single(cls) -> "TPContext":
        return cls()

    @classmethod
    def from_group(cls, group=None) -> "TPContext":
        return cls(dist.get_rank(group), dist.get_world_size(group), group)

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return x
        if self.fast_allreduce is not None:
            y = self.fast_allreduce(x)
            if y is not None:
                return y
        dist.all_reduce(x, group=self.group)
        return x

    def all_reduce_async(self, x: torch.Tensor):
        """Start a sum all-reduce without blocking the compute stream; returns (x, work) — call ``work.wait()`` before
        reading x (on GPU that makes the current HIP stream wait for RCCL's stream, nothing blocks on the host)."""
        if self.world == 1:
            return x, None
        return x, dist.all_reduce(x, group=self.group, async_op=True)

    def enable_ipc_allreduce(self, max_bytes: int = 8 << 20, threshold: int = 4 << 20):
        """Route bf16 all-reduces of at most ``threshold`` bytes to the IPC kernels (K14: one-shot for small messages,
        two-shot above ``IpcAllReduce.two_shot_min_bytes`` at W > 2); larger messages (prefill chunks), where RCCL's
        multi-channel rings use the links best, stay on RCCL."""
        from .custom_ar import IpcAllReduce

        ar = IpcAllReduce(self.group, max_bytes)

        def fast(x: torch.Tensor) -> Optional[torch.Tensor]:
            if x.numel() * x.element_size() <= threshold and ar.fits(x) and x.is_contiguous():
                return ar.all_reduce(x, out=x)
            return None

        def fast_norm(x: torch.Tensor, resid: torch.Tensor, w: torch.Tensor, eps: float) -> Optional[torch.Tensor]:
            # the fused kernel is one-shot (every rank reads all W peers' rows): messages the size policy sends to
            # two-shot (mid-sized, W > 2) take the two-shot all-reduce + add_rmsnorm instead
            if (x.numel() * x.element_size() <= threshold and ar.fits(x) and x.dim() == 2 and x.is_contiguous()
                    and resid.is_contiguous() and x.shape[1] % 8 == 0 and x.shape[1] <= 16384 and ar.pick(x) == 1):
                return ar.all_reduce_norm(x, resid, w, eps)
            return None

        self.fast_allreduce = fast
        self.fast_allreduce_norm = fast_norm
        self.ipc_allreduce = ar
        return ar

    def all_reduce_add_rmsnorm(self, x: torch.Tensor, resid: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
        """resid <- bf16(sum over ranks of x + resid) in place; returns rmsnorm(resid) * w.  One launch on the fused
        IPC kernel (K14 + residual + RMSNorm) when it takes the message, else all-reduce then ops.add_rmsnorm."""
        if self.fast_allreduce_norm is not None:
            y = self.fast_allreduce_norm(x, resid, w, eps)
            if y is not None:
                return y
        from .. import ops

        return ops.add_rmsnorm(self.all_reduce(x), resid, w, eps)

    def reduce_scatter_rows(self, x: torch.Tensor) -> torch.Tensor:
        """Sequence parallelism: sum over ranks of x [R * world, ...], this rank keeping rows [rank * R, (rank + 1) * R)
        (RCCL reduce-scatter: the same bytes on the wire as half an all-reduce)."""
        if self.world == 1:
            return x
        out = torch.empty((x.shape[0] // self.world,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.reduce_scatter_tensor(out, x.contiguous(), group=self.group)
        return out

    def all_gather_rows(self, x: torch.Tensor) -> torch.Tensor:
        """Sequence parallelism: [R, ...] row shards -> [R * world, ...] in rank order."""
        if self.world == 1:
            return x
        out = torch.empty((x.shape[0] * self.world,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x.contiguous(), group=self.group)
        return out

    def all_gather_last(self, x: torch.Tensor) -> torch.Tensor:
        """[.., n] shards -> [.., n * world] (vocab-parallel logits)."""
        if self.world == 1:
            return x
        parts = [torch.empty_like(x) for _ in range(self.world)]
        dist.all_gather(parts, x.contiguous(), group=self.group)
        return torch.cat(parts, dim=-1)

    def broadcast_obj(self, obj, src: int = 0):
        if self.world == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src, group=self.group)
        return box[0]
