"""Host-side mirror of the reference's filter classes, running on the HIP path.

Same names, argument meaning and error behaviour as:
  FullFilterBlockBuilder  table/full_filter_block.h:33-70, .cc:16-147
  FullFilterBlockReader   table/full_filter_block.h:71-94, .cc:186-294
  BloomFilterPolicy       include/TimberSaw/filter_policy.h:31-71, util/bloom.cc:14-91

Differences, all deliberate:
  * Corrupt full-filter metadata raises DlsmError(DLSM_E_CORRUPT) where the
    reference prints and exit(1)s (full_filter_block.cc:216-249).
  * ``AddKeys`` / ``KeysMayMatch`` are batch forms (the reference has no
    MultiGet, TODO:8); they are what the GPU is for.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from . import Context, Keys, full_parse, lib
from ._lib import DLSM_OK, DlsmError

NAME = "TimberSaw.BuiltinBloomFilter2"  # util/bloom.cc:23 -- the format identity


class FullFilterBlockBuilder:
    """FullFilterBlockBuilder(ibv_mr* mr, int bits_per_key).

    ``slot`` is the caller-owned output buffer (the reference's RDMA-registered
    FilterChunk slot, zeroed by every reference caller); a writable uint8 numpy
    array.  After ``Finish()``, ``result`` is a memoryview of the filter bytes
    inside the slot.  The call order is ``(RestartBlock AddKey*)* Finish``.
    """

    def __init__(self, slot: np.ndarray, bits_per_key: int, ctx: Context):
        self.local_mr = slot
        self.bits_per_key_ = bits_per_key
        self.num_probes_ = int(lib().dlsm_bloom_full_num_probes(bits_per_key))
        self.ctx = ctx
        self._target = slot
        self.result = memoryview(slot)[:0]
        self._keys: list[bytes] = []
        self._batches: list[Keys] = []

    def RestartBlock(self, block_offset: int = 0) -> None:
        # full_filter_block.cc:30-33: clears pending hashes
        self._keys.clear()
        self._batches.clear()

    def AddKey(self, key: bytes) -> None:
        self._keys.append(bytes(key))

    def AddKeys(self, keys: Keys) -> None:
        """Append a packed batch of keys in table order (host memory)."""
        if self._keys:
            self._batches.append(Keys.pack(self._keys))
            self._keys = []
        self._batches.append(keys)

    def _pending(self) -> Keys:
        if self._keys:
            self._batches.append(Keys.pack(self._keys))
            self._keys = []
        if not self._batches:
            return Keys(np.zeros(16, np.uint8), 0, 0, None)
        if len(self._batches) == 1:
            return self._batches[0]
        parts = []
        for b in self._batches:
            if b.offsets is None:
                parts += [bytes(b.data[i * b.key_len:(i + 1) * b.key_len]) for i in range(b.n)]
            else:
                parts += [bytes(b.data[int(b.offsets[i]):int(b.offsets[i + 1])]) for i in range(b.n)]
        return Keys.pack(parts)

    def Finish(self) -> None:
        keys = self._pending()
        out = self._target
        cap = out.size
        flt = self.ctx.full_build([keys], self.bits_per_key_, caps=[cap])[0]
        out[: len(flt)] = np.frombuffer(flt, dtype=np.uint8)
        self._batches.clear()
        self.result = memoryview(out)[: len(flt)]

    def Reset(self) -> None:
        self._target = self.local_mr
        self.result = memoryview(self.local_mr)[:0]

    def Move_buffer(self, p: np.ndarray) -> None:
        self._target = p
        self.result = memoryview(p)[:0]


class FullFilterBlockReader:
    """FullFilterBlockReader(const Slice& contents, rdma_mg, side)."""

    def __init__(self, contents: bytes, ctx: Context):
        self.filter_content = bytes(contents)
        st, k, L, lg = full_parse(self.filter_content)
        if st != DLSM_OK:
            raise DlsmError(st, "FullFilterBlockReader")
        self.num_probes_, self.num_lines_, self.log2_cache_line_size_ = k, L, lg
        self.ctx = ctx
        self._fs = ctx.filterset([self.filter_content])

    def KeyMayMatch(self, key: bytes) -> bool:
        return bool(self.KeysMayMatch(Keys.pack([bytes(key)]))[0])

    def KeysMayMatch(self, keys: Keys) -> np.ndarray:
        return self.ctx.full_probe(self._fs, keys).astype(bool)


class BloomFilterPolicy:
    """NewBloomFilterPolicy(bits_per_key) -- the legacy FilterPolicy format."""

    def __init__(self, bits_per_key: int, ctx: Context):
        self.bits_per_key_ = bits_per_key
        self.ctx = ctx

    def Name(self) -> str:
        return NAME

    def CreateFilter(self, keys: Sequence[bytes], n: int, dst: bytearray) -> None:
        """Append a filter summarising keys[0, n) to dst (util/bloom.cc:25-55)."""
        flt = self.ctx.legacy_build([Keys.pack([bytes(k) for k in keys[:n]])], self.bits_per_key_)[0]
        dst += flt

    def KeyMayMatch(self, key: bytes, bloom_filter: bytes) -> bool:
        return bool(self.ctx.legacy_probe(bytes(bloom_filter), Keys.pack([bytes(key)]))[0])

    def KeysMayMatch(self, keys: Keys, bloom_filter: bytes) -> np.ndarray:
        return self.ctx.legacy_probe(bytes(bloom_filter), keys).astype(bool)
