"""Paged KV-cache block allocator.

Block ids index the per-layer cache tensors ``k_cache[nb, nkv, bs, d]`` /
``v_cache[nb, nkv, bs/8, d, 8]``.  Block 0 is reserved (never handed out) so padded
block-table entries always point at valid memory.  Each running sequence owns a
row ("slot") of a persistent int32 block table that is updated incrementally as
blocks are appended, so building a step's block tables is a single row gather.
Sized for 288 GB HBM: block tables are int32 (up to 2^31 blocks) and the free
list is a plain Python list used as a stack (O(1) alloc/free).
"""
from __future__ import annotations

import numpy as np

from .sequence import Sequence


class BlockManager:
    def __init__(self, num_blocks: int, block_size: int, max_seqs: int, max_blocks_per_seq: int,
                 watermark: float = 0.01):
        assert num_blocks >= 2, "need at least 2 KV blocks"
        self.num_blocks = num_blocks
        self.block_size = block_size
        self.max_blocks_per_seq = max_blocks_per_seq
        self.free: list[int] = list(range(num_blocks - 1, 0, -1))   # block 0 reserved
        self.watermark = max(1, int(watermark * num_blocks))
        self.table = np.zeros((max_seqs, max_blocks_per_seq), dtype=np.int32)
        self.free_slots: list[int] = list(range(max_seqs - 1, -1, -1))

    @property
    def num_free(self) -> int:
        return len(self.free)

    def usage(self) -> float:
        return 1.0 - len(self.free) / max(1, self.num_blocks - 1)

    def blocks_needed(self, seq: Sequence, num_tokens: int) -> int:
        need = -(-num_tokens // self.block_size)
        return max(0, need - len(seq.block_ids))

    def can_allocate(self, seq: Sequence, num_tokens: int, watermark: bool = False) -> bool:
        need = self.blocks_needed(seq, num_tokens)
        if -(-num_tokens // self.block_size) > self.max_blocks_per_seq:
            return False
        return need + (self.watermark if watermark else 0) <= len(self.free)

    def allocate(self, seq: Sequence, num_tokens: int) -> None:
        """Grow seq's block list to cover num_tokens tokens (caller checked capacity)."""
        if seq.slot < 0:
            seq.slot = self.free_slots.pop()
        need = self.blocks_needed(seq, num_tokens)
        row = self.table[seq.slot]
        for _ in range(need):
            b = self.free.pop()
            row[len(seq.block_ids)] = b
            seq.block_ids.append(b)

    def free_seq(self, seq: Sequence) -> None:
        self.free.extend(reversed(seq.block_ids))
        if seq.slot >= 0:
            self.table[seq.slot, : len(seq.block_ids)] = 0
            self.free_slots.append(seq.slot)
            seq.slot = -1
        seq.block_ids = []

    def check_invariants(self, seqs=()) -> None:
        """Debug (KGC_DEBUG=1 checks this every engine step): no block is both free and
        owned or owned twice; block 0 is never handed out; every block is accounted
        for; each owner's block-table row mirrors its block list."""
        fs = set(self.free)
        assert len(fs) == len(self.free), "duplicate free block"
        assert 0 not in fs, "reserved block 0 on the free list"
        owned: set = set()
        for s in seqs:
            if not s.block_ids:
                continue
            b = set(s.block_ids)
            assert len(b) == len(s.block_ids), f"{s.request_id} holds a block twice"
            assert 0 not in b, f"{s.request_id} holds reserved block 0"
            assert not (b & fs), f"{s.request_id} holds a free block"
            assert not (b & owned), f"{s.request_id} shares a block with another sequence"
            owned |= b
            assert s.slot >= 0, f"{s.request_id} owns blocks but no table slot"
            row = self.table[s.slot, : len(s.block_ids)]
            assert row.tolist() == s.block_ids, f"{s.request_id} block-table row is stale"
        if seqs:
            assert len(owned) + len(fs) == self.num_blocks - 1, "leaked KV blocks"
