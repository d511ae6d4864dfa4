"""Paged-KV block allocator with automatic prefix caching (SURVEY.md §1.2 N4, §5.7 "prefix caching of the fixed
prompt template").

Every CHRONOS prompt starts with the same Llama-3 chat header + "Analyze this sequence. Return JSON ONLY.\\n
Sequence: [" (chronos_sensor.py:109-111): one full 16-token KV block that every chain would otherwise recompute.
Full blocks of prompt tokens are content-addressed by a chained SHA-256 digest (parent digest, token ids); a new
request reuses
the longest cached run of its prompt's full blocks (refcounted, read-only) and prefills only the remainder.  Blocks
whose refcount drops to zero stay cached and are recycled least-recently-used when the free list runs dry.

Partial blocks: a prompt whose next block matches a cached block (full, or the partial last block of another prompt)
only for its first j < 16 tokens gets a fresh block with those j computed token slots copied in (``lookup_partial``;
the engine batches the copies before its next prefill forward) and prefills from token j.  Without it every prompt
recomputes up to 15 tokens of its shared prefix: the wave's prompts share ~47 of ~93 tokens, ending mid-block.
A source qualifies only for slots a launched prefill has already written (``mark_computed``), so the stream-ordered
copy reads finished K/V.

Block 0 is reserved as a scratch block: empty decode slots point their block table at it, so a captured decode graph
that always runs a fixed number of rows never writes into another sequence's KV.
"""
from __future__ import annotations

import hashlib
from array import array
from collections import OrderedDict
from typing import Sequence


class BlockManager:
    def __init__(self, num_blocks: int, block_size: int, prefix_cache: bool = True, partial_prefix: bool = True):
        if num_blocks < 2:
            raise ValueError("need at least 2 KV blocks (block 0 is scratch)")
        self.num_blocks, self.block_size = num_blocks, block_size
        self.prefix_cache = prefix_cache
        self.partial_prefix = prefix_cache and partial_prefix
        self._free = list(range(num_blocks - 1, 0, -1))
        self._ref: dict[int, int] = {}
        self._by_hash: dict[bytes, int] = {}     # content digest -> block
        self._hash_of: dict[int, bytes] = {}     # block -> content digest
        self._evictable: "OrderedDict[int, None]" = OrderedDict()  # cached blocks with refcount 0 (LRU order)
        # partial-block sources: parent digest -> blocks at that depth; block -> (parent digest, its prompt tokens,
        # computed slots).  An entry lives while its block holds that content: _drop_part removes it from both maps
        # when the block is reused or freed, so neither grows past the number of blocks (argv makes most parents
        # unique per prompt, and such a parent is never looked up again).
        self._children: dict[bytes, dict[int, None]] = {}
        self._part: dict[int, list] = {}
        self._memo = None  # (tokens, len, digest chain) of the last prompt hashed
        self.hits = 0
        self.lookups = 0

    def blocks_for(self, tokens: int) -> int:
        return (tokens + self.block_size - 1) // self.block_size

    @property
    def free(self) -> int:
        return len(self._free) + len(self._evictable)

    def can_alloc(self, n: int) -> bool:
        return self.free >= n

    def _drop_part(self, b: int) -> None:
        e = self._part.pop(b, None)
        if e is not None:
            kids = self._children.get(e[0])
            if kids is not None:
                kids.pop(b, None)
                if not kids:
                    del self._children[e[0]]

    def _take(self) -> int:
        if self._free:
            b = self._free.pop()
        else:
            b, _ = self._evictable.popitem(last=False)  # least recently used cached block
            h = self._hash_of.pop(b)
            self._by_hash.pop(h, None)
        self._drop_part(b)  # new content: no longer a partial-block source
        return b

    def alloc(self, n: int) -> list[int]:
        if n > self.free:
            raise MemoryError(f"KV cache exhausted: want {n} blocks, {self.free} free")
        out = [self._take() for _ in range(n)]
        for b in out:
            self._ref[b] = 1
        return out

    def release(self, blocks: Sequence[int]) -> None:
        for b in blocks:
            r = self._ref.get(b, 0) - 1
            if r > 0:
                self._ref[b] = r
                continue
            self._ref.pop(b, None)
            if b in self._hash_of:
                self._evictable[b] = None
            else:
                self._drop_part(b)
                self._free.append(b)

    # ---- prefix cache ----------------------------------------------------------------------------------------------
    def _hashes(self, tokens: Sequence[int], nblocks: int) -> list[bytes]:
        """Chained SHA-256 digests (parent digest || block token ids as int32).  Prompt tokens are partly
        attacker-controlled (argv paths in the telemetry), so the key must be collision-resistant: a 64-bit
        non-cryptographic hash collision would hand one prompt another prompt's KV block."""
        # Admission asks for the same prompt's chain up to four times (lookup, lookup_partial, register,
        # note_prompt): keep the last prompt's full chain (identity-checked, the object is held so its id stays
        # unique).
        m = self._memo
        if m is not None and m[0] is tokens and m[1] == len(tokens) and len(m[2]) >= nblocks:
            return m[2][:nblocks]
        hs, h = [], b""
        bs = self.block_size
        for i in range(max(nblocks, len(tokens) // bs)):
            h = hashlib.sha256(h + array("i", tokens[i * bs:(i + 1) * bs]).tobytes()).digest()
            hs.append(h)
        self._memo = (tokens, len(tokens), hs)
        return hs[:nblocks]

    def lookup(self, tokens: Sequence[int]) -> list[int]:
        """Longest run of cached full blocks at the start of `tokens` (never the whole prompt: the last token must be
        recomputed for its logits).  The returned blocks are referenced for the caller."""
        if not self.prefix_cache:
            return []
        self.lookups += 1
        n = (len(tokens) - 1) // self.block_size
        out = []
        for h in self._hashes(tokens, n):
            b = self._by_hash.get(h)
            if b is None:
                break
            out.append(b)
        for b in out:
            if b in self._evictable:
                del self._evictable[b]
            self._ref[b] = self._ref.get(b, 0) + 1
        self.hits += bool(out)
        return out

    def register(self, tokens: Sequence[int], blocks: Sequence[int]) -> None:
        """After a prompt's KV is written: publish its full blocks for reuse."""
        if not self.prefix_cache:
            return
        n = min(len(tokens) // self.block_size, len(blocks))
        for h, b in zip(self._hashes(tokens, n), blocks[:n]):
            if h in self._by_hash or b in self._hash_of:
                continue
            self._by_hash[h] = b
            self._hash_of[b] = h

    def note_prompt(self, tokens: Sequence[int], blocks: Sequence[int], first: int = 0) -> None:
        """Record blocks[first:] of a prompt as future partial-block sources (no slot computed yet)."""
        if not self.partial_prefix:
            return
        bs = self.block_size
        n = min(self.blocks_for(len(tokens)), len(blocks))
        hs = [b""] + self._hashes(tokens, n - 1)
        for d in range(first, n):
            b = blocks[d]
            if b in self._part:
                continue
            self._part[b] = [hs[d], tuple(tokens[d * bs:(d + 1) * bs]), 0]
            self._children.setdefault(hs[d], {})[b] = None

    def mark_computed(self, blocks: Sequence[int], start: int, end: int) -> None:
        """Token positions [start, end) of the sequence owning ``blocks`` now have their K/V written (in stream
        order)."""
        bs = self.block_size
        for d in range(start // bs, min(len(blocks), (end + bs - 1) // bs)):
            e = self._part.get(blocks[d])
            if e is not None and max(0, start - d * bs) <= e[2]:  # keeps the computed slots contiguous from 0
                e[2] = max(e[2], min(bs, end - d * bs))

    def lookup_partial(self, tokens: Sequence[int], nfull: int, min_tokens: int = 2):
        """After ``nfull`` shared full blocks: the computed block at depth ``nfull`` whose slots agree longest with
        the prompt's next tokens -> (block, j), the block referenced for the caller (release it once copied);
        None below ``min_tokens``.  Never the whole prompt: its last token is recomputed for the logits."""
        if not self.partial_prefix:
            return None
        bs = self.block_size
        parent = self._hashes(tokens, nfull)[-1] if nfull else b""
        want = tokens[nfull * bs:(nfull + 1) * bs]
        cap = min(len(want), len(tokens) - 1 - nfull * bs)
        best, bj = None, min_tokens - 1
        for b in self._children.get(parent, ()):
            e = self._part[b]
            lim = min(cap, e[2])
            j = 0
            toks = e[1]
            while j < lim and j < len(toks) and toks[j] == want[j]:
                j += 1
            if j > bj:
                best, bj = b, j
        if best is None:
            return None
        if best in self._evictable:
            del self._evictable[best]
        self._ref[best] = self._ref.get(best, 0) + 1
        return best, bj

    def clear_cache(self) -> None:
        """Forget every cached prefix (blocks still referenced keep their contents; idle cached blocks are freed)."""
        for b in list(self._evictable):
            self._free.append(b)
        self._evictable.clear()
        self._by_hash.clear()
        self._hash_of.clear()
        self._children.clear()
        self._part.clear()

    def usage(self) -> float:
        return 1.0 - self.free / (self.num_blocks - 1)
