"""Paged KV-cache block allocator with automatic prefix caching.

Block ids index the per-layer cache tensors ``k_cache[nb, nkv, bs, d]`` /
``v_cache[nb, nkv, bs/8, d, 8]``.
- Block 0 is reserved (never handed out), so padded block-table entries always point at valid memory.
- Each running sequence owns a row ("slot") of a persistent int32 block table. The row is updated incrementally as blocks are appended, so building a step's block tables is a single row gather.
- Sized for 288 GB HBM: block tables are int32 (up to 2^31 blocks), and the free list is a stack (O(1) allocate/free).

Prefix caching (vLLM's automatic prefix caching, on by default in its V1 engine):
- A FULL block whose token ids are all known is content-addressed. Its key is a 128-bit
  keyed BLAKE2b of (parent block's key, its block_size token ids), so one key names a whole
  prefix. The BLAKE2b key is a random per-process salt: keys cannot be precomputed by a
  client, unlike Python's unseeded ``hash()`` of an int tuple (the vLLM CVE-2025-25183 class).
- A hit is verified, not trusted: every cached block keeps its parent key and token ids, and
  a lookup whose stored (parent key, tokens) differ from the sequence's stops there and the
  rest of the prompt is recomputed.
- Blocks are reference counted.
  - A sequence admitted with a prompt whose leading full blocks are cached takes references on those blocks. It starts computing after them, and the prefill kernel reads them as context, exactly like a chunked-prefill continuation.
  - A block whose last reference goes away keeps its contents and its key. It moves to an LRU list of evictable blocks.
  - Allocation takes never-cached blocks first, then evicts the least-recently-freed cached block.
- A recompute-preempted sequence re-admitted later usually finds its own blocks still cached.
"""
from __future__ import annotations

import collections
import hashlib
import os

import numpy as np

from .sequence import Sequence


class BlockManager:
    def __init__(self, num_blocks: int, block_size: int, max_seqs: int, max_blocks_per_seq: int,
                 watermark: float = 0.01, enable_prefix_caching: bool = False):
        assert num_blocks >= 2, "need at least 2 KV blocks"
        self.num_blocks = num_blocks
        self.block_size = block_size
        self.max_blocks_per_seq = max_blocks_per_seq
        self.free: list[int] = list(range(num_blocks - 1, 0, -1))   # block 0 reserved
        self.watermark = max(1, int(watermark * num_blocks))
        self.table = np.zeros((max_seqs, max_blocks_per_seq), dtype=np.int32)
        self.free_slots: list[int] = list(range(max_seqs - 1, -1, -1))
        self.prefix_caching = enable_prefix_caching
        self.ref = np.zeros(num_blocks, dtype=np.int32) if enable_prefix_caching else None
        self.key_of: dict[int, bytes] = {}                     # cached block -> prefix key
        self.block_of: dict[bytes, int] = {}                   # prefix key -> cached block
        self.content_of: dict[int, tuple] = {}                 # cached block -> (parent key, toks)
        self._salt = os.urandom(16)
        self.evictable: collections.OrderedDict[int, None] = collections.OrderedDict()
        self.hit_tokens = 0                                    # prefix-cache statistics
        self.query_tokens = 0
        self.collisions = 0

    # ---------------------------------------------------------------- capacity
    @property
    def num_free(self) -> int:
        return len(self.free) + len(self.evictable)

    def usage(self) -> float:
        return 1.0 - self.num_free / max(1, self.num_blocks - 1)

    def blocks_needed(self, seq: Sequence, num_tokens: int) -> int:
        need = -(-num_tokens // self.block_size)
        return max(0, need - len(seq.block_ids))

    def can_allocate(self, seq: Sequence, num_tokens: int, watermark: bool = False) -> bool:
        need = self.blocks_needed(seq, num_tokens)
        if -(-num_tokens // self.block_size) > self.max_blocks_per_seq:
            return False
        return need + (self.watermark if watermark else 0) <= self.num_free

    # ---------------------------------------------------------------- allocation
    def _take_block(self) -> int:
        if self.free:
            return self.free.pop()
        b, _ = self.evictable.popitem(last=False)          # least recently freed
        key = self.key_of.pop(b)
        self.content_of.pop(b, None)
        if self.block_of.get(key) == b:
            del self.block_of[key]
        return b

    def _slot(self, seq: Sequence) -> None:
        if seq.slot < 0:
            seq.slot = self.free_slots.pop()

    def allocate(self, seq: Sequence, num_tokens: int) -> None:
        """Grow seq's block list to cover num_tokens tokens (caller checked capacity)."""
        self._slot(seq)
        need = self.blocks_needed(seq, num_tokens)
        row = self.table[seq.slot]
        for _ in range(need):
            b = self._take_block()
            if self.ref is not None:
                self.ref[b] = 1
            row[len(seq.block_ids)] = b
            seq.block_ids.append(b)

    def free_seq(self, seq: Sequence) -> None:
        if self.ref is None:
            self.free.extend(reversed(seq.block_ids))
        else:
            for b in reversed(seq.block_ids):
                self.ref[b] -= 1
                if self.ref[b] == 0:
                    if b in self.key_of:
                        self.evictable[b] = None            # keep contents for reuse
                    else:
                        self.free.append(b)
        if seq.slot >= 0:
            self.table[seq.slot, : len(seq.block_ids)] = 0
            self.free_slots.append(seq.slot)
            seq.slot = -1
        seq.block_ids = []
        seq.num_registered = 0

    # ---------------------------------------------------------------- prefix caching
    def block_key(self, parent: bytes, toks) -> bytes:
        h = hashlib.blake2b(parent, digest_size=16, key=self._salt)
        h.update(np.asarray(toks, dtype=np.int64).tobytes())
        return h.digest()

    def _keys(self, seq: Sequence, n_full: int) -> list[bytes]:
        """Prefix keys of seq's first n_full blocks (memoised on the sequence; its token
        ids never change, so the keys stay valid across preemptions)."""
        keys = seq.block_keys
        bs = self.block_size
        while len(keys) < n_full:
            i = len(keys)
            toks = seq.tokens_slice(i * bs, (i + 1) * bs)
            keys.append(self.block_key(keys[-1] if keys else b"", toks))
        return keys[:n_full]

    def cached_prefix_blocks(self, seq: Sequence) -> list[int]:
        """Leading full blocks of a waiting sequence's tokens that are cached.  At least
        one token is always left to compute (the sampled position needs logits)."""
        if self.ref is None or seq.block_ids:
            return []
        # never key over a token id still pending on the GPU
        n_full = min(seq.num_tokens - 1, seq.num_tokens - seq.num_pending) // self.block_size
        hits = []
        bs = self.block_size
        keys = self._keys(seq, n_full)
        for i, key in enumerate(keys):
            b = self.block_of.get(key)
            if b is None:
                break
            parent = keys[i - 1] if i else b""
            if self.content_of.get(b) != (parent, tuple(seq.tokens_slice(i * bs, (i + 1) * bs))):
                self.collisions += 1          # key matched, content did not: recompute
                break
            hits.append(b)
        return hits

    def can_admit(self, seq: Sequence, num_tokens: int, hits: list[int]) -> bool:
        """can_allocate(..., watermark=True) for a sequence that will first take the
        cached blocks ``hits`` (evictable hits leave the free pool)."""
        total = -(-num_tokens // self.block_size)
        if total > self.max_blocks_per_seq:
            return False
        taken = sum(1 for b in hits if b in self.evictable)
        return max(0, total - len(hits)) + self.watermark <= self.num_free - taken

    def take_prefix(self, seq: Sequence, hits: list[int]) -> int:
        """Attach the cached blocks to seq; returns the number of cached tokens."""
        self._slot(seq)
        row = self.table[seq.slot]
        for b in hits:
            if self.ref[b] == 0:
                self.evictable.pop(b, None)
            self.ref[b] += 1
            row[len(seq.block_ids)] = b
            seq.block_ids.append(b)
        seq.num_registered = len(hits)
        n = len(hits) * self.block_size
        self.hit_tokens += n
        return n

    def note_query(self, seq: Sequence) -> None:
        self.query_tokens += seq.num_tokens

    def register_full_blocks(self, seq: Sequence, num_known: int) -> None:
        """Publish seq's blocks that are full of computed tokens whose ids are known
        (``num_known`` leading token ids are final, i.e. not still pending on the GPU)."""
        if self.ref is None or seq.slot < 0:
            return
        n_full = min(seq.num_computed, num_known, len(seq.block_ids) * self.block_size)
        n_full //= self.block_size
        if n_full <= seq.num_registered:
            return
        keys = self._keys(seq, n_full)
        bs = self.block_size
        for i in range(seq.num_registered, n_full):
            b = seq.block_ids[i]
            if b in self.key_of or keys[i] in self.block_of:
                continue        # a prefix hit (already published), or the same content elsewhere
            self.key_of[b] = keys[i]
            self.block_of[keys[i]] = b
            self.content_of[b] = (keys[i - 1] if i else b"",
                                  tuple(seq.tokens_slice(i * bs, (i + 1) * bs)))
        seq.num_registered = n_full

    def hit_rate(self) -> float:
        return self.hit_tokens / self.query_tokens if self.query_tokens else 0.0

    # ---------------------------------------------------------------- debug
    def check_invariants(self, seqs=()) -> None:
        """Debug (KGC_DEBUG=1 checks this every engine step).
        - Block 0 is never handed out.
        - Every block is exactly one of: free, evictable (cached, unreferenced), or held.
        - A held block's refcount is the number of sequences holding it.
        - Each holder's block-table row mirrors its block list.
        Without prefix caching a block has at most one holder."""
        fs = set(self.free)
        assert len(fs) == len(self.free), "duplicate free block"
        assert 0 not in fs, "reserved block 0 on the free list"
        ev = set(self.evictable)
        assert not (fs & ev), "block both free and evictable"
        holders: collections.Counter = collections.Counter()
        for s in seqs:
            if not s.block_ids:
                continue
            b = set(s.block_ids)
            assert len(b) == len(s.block_ids), f"{s.request_id} holds a block twice"
            assert 0 not in b, f"{s.request_id} holds reserved block 0"
            assert not (b & fs), f"{s.request_id} holds a free block"
            assert not (b & ev), f"{s.request_id} holds an evictable block"
            assert s.slot >= 0, f"{s.request_id} owns blocks but no table slot"
            row = self.table[s.slot, : len(s.block_ids)]
            assert row.tolist() == s.block_ids, f"{s.request_id} block-table row is stale"
            holders.update(b)
        if self.ref is None:
            assert all(c == 1 for c in holders.values()), "a block is shared without prefix caching"
        else:
            for b, c in holders.items():
                assert self.ref[b] == c, f"block {b}: refcount {self.ref[b]} != {c} holders"
            for b in ev:
                assert self.ref[b] == 0 and b in self.key_of, f"evictable block {b} is referenced"
        if seqs:
            assert len(holders) + len(fs) + len(ev) == self.num_blocks - 1, "leaked KV blocks"
