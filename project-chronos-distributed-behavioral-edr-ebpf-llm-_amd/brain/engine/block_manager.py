"""Paged-KV block allocator.

Block 0 is reserved as a scratch block: empty decode slots point their block table at it, so a captured decode graph
that always runs a fixed number of rows never writes into another sequence's KV.
"""
from __future__ import annotations


class BlockManager:
    def __init__(self, num_blocks: int, block_size: int):
        if num_blocks < 2:
            raise ValueError("need at least 2 KV blocks (block 0 is scratch)")
        self.num_blocks, self.block_size = num_blocks, block_size
        self._free = list(range(num_blocks - 1, 0, -1))

    def blocks_for(self, tokens: int) -> int:
        return (tokens + self.block_size - 1) // self.block_size

    @property
    def free(self) -> int:
        return len(self._free)

    def can_alloc(self, n: int) -> bool:
        return len(self._free) >= n

    def alloc(self, n: int) -> list[int]:
        if n > len(self._free):
            raise MemoryError(f"KV cache exhausted: want {n} blocks, {len(self._free)} free")
        out = self._free[-n:][::-1] if n else []
        del self._free[len(self._free) - n:]
        return out

    def release(self, blocks: list[int]) -> None:
        self._free.extend(reversed(blocks))

    def usage(self) -> float:
        return 1.0 - len(self._free) / (self.num_blocks - 1)
