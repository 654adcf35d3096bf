"""The host's copy of the pushed rows, kept by sequence number, and the compact match decoders.

Python mirror of the Java binding's ``ColumnarBatch`` history and ``GpuStateStreamRuntime``'s
record decoding (java/.../state/gpu/), so the rules the Java side follows are executed and tested
here (there is no JDK in this image):

* **Retention by sequence number.**  The engine names a match's events by sequence number; the host
  rebuilds the ``StreamEvent`` of each from its own copy of the row.  The reference keeps a
  ``StreamEvent`` alive exactly as long as a partial holds it (``StreamPreStateProcessor.java:
  364-403``: the partial sits on the pending list with its events until it matches or expires).  The
  host keeps every row from ``shp_engine_oldest_live_seq`` on (the oldest event an open partial of the
  engine's committed state holds); a later push's matches name only those rows and its own.  Trims
  are amortised: the engine is asked only when the kept rows have doubled since the last trim (and
  at least ``min_trim`` are kept), so its cost (a state snapshot) stays a fraction of the rows'.
* **PAIRS32** (sweep path): word pair ``(e2's index in the pushed batch, e2 seq - e1 seq)``.
* **CHAIN32** (count-sequence path): word ``e2's index | L << 28``; e1's chain is the L events of
  e2's partition key just before e2 (a sequence keeps them consecutive), tracked per key in a ring
  of the key's last M sequence numbers as the batch's rows are walked in order.

Both compact forms come back per key in emission order but across keys in owner order; the
reference emits at e2's arrival (``PatternSingleProcessStreamReceiver`` /
``SequenceSingleProcessStreamReceiver`` run the chain per event), so the host restores the global
order with a stable sort on e2's batch index.
"""
from __future__ import annotations

from collections import deque
from typing import Dict, List, Tuple

import numpy as np

CH32_LEN_SHIFT = 28
CH32_IDX_MASK = (1 << CH32_LEN_SHIFT) - 1


class EvictedRow(LookupError):
    """A match named a row the history no longer holds (a retention bug, never expected)."""


class RowHistory:
    """Rows by sequence number, in blocks of one push each: (seq0, rows)."""

    def __init__(self, min_trim: int = 4096):
        self.seq0: deque = deque()
        self.blocks: deque = deque()
        self.next_seq = 0
        self.kept = 0
        self.min_trim = max(1, int(min_trim))
        self.trim_at = self.min_trim
        self.floor = 0          # every row below this was dropped
        self.trims = 0          # oldest-live queries made
        self.dropped = 0

    def add_block(self, rows: List[tuple]) -> int:
        """The rows of one successful push; returns the block's first sequence number."""
        s0 = self.next_seq
        if rows:
            self.seq0.append(s0)
            self.blocks.append(rows)
            self.next_seq += len(rows)
            self.kept += len(rows)
        return s0

    def __getitem__(self, seq: int):
        if seq < self.floor or seq >= self.next_seq:
            raise EvictedRow(f"event {seq} is not held (kept [{self.floor}, {self.next_seq}))")
        i = self._find(seq)
        return self.blocks[i][seq - self.seq0[i]]

    def _find(self, seq: int) -> int:
        # deque has no bisect support: binary search over its indices
        lo, hi = 0, len(self.seq0) - 1
        while lo < hi:
            mid = (lo + hi + 1) // 2
            if self.seq0[mid] <= seq:
                lo = mid
            else:
                hi = mid - 1
        return lo

    def maybe_trim(self, oldest_live) -> bool:
        """Drop the rows below the engine's oldest live sequence number once the kept rows have
        doubled since the last trim.  oldest_live: a callable (shp_engine_oldest_live_seq)."""
        if self.kept < self.trim_at:
            return False
        lo = int(oldest_live())
        self.trims += 1
        self.trim_below(lo)
        self.trim_at = max(self.min_trim, 2 * self.kept)
        return True

    def trim_below(self, lo: int):
        while self.blocks and self.seq0[0] + len(self.blocks[0]) <= lo:
            n = len(self.blocks[0])
            self.blocks.popleft()
            self.seq0.popleft()
            self.kept -= n
            self.dropped += n
        if self.blocks and self.seq0[0] < lo:  # a push partly below: keep its live tail
            cut = lo - self.seq0[0]
            self.blocks[0] = self.blocks[0][cut:]
            self.seq0[0] = lo
            self.kept -= cut
            self.dropped += cut
        self.floor = max(self.floor, min(lo, self.next_seq))


def decode_pairs32(words: np.ndarray, seq0: int) -> List[Tuple[int, List[List[int]]]]:
    """PAIRS32 words -> [(e2's batch index, [[e1 seq], [e2 seq]])] in the reference's global
    emission order (stable by e2's index: the engine's per-key order is kept)."""
    w = np.asarray(words, np.uint32).reshape(-1, 2)
    idx = w[:, 0].astype(np.int64)
    order = np.argsort(idx, kind="stable")
    out = []
    for j in order:
        e2 = seq0 + int(idx[j])
        out.append((int(idx[j]), [[e2 - int(w[j, 1])], [e2]]))
    return out


class ChainRings:
    """Per partition key, the sequence numbers of its last M events (CHAIN32 decoding)."""

    def __init__(self, M: int):
        self.M = M
        self.rings: Dict[int, deque] = {}

    def decode(self, words: np.ndarray, keys: np.ndarray, counted: np.ndarray, seq0: int):
        """CHAIN32 words of one push -> [(e2's batch index, [e1 chain, [e2 seq]])] in batch order.
        keys: the push's key ids; counted: rows the sequence counts per key (rows of the query's
        stream -- clock-only rows are not events of any key)."""
        w = np.asarray(words, np.uint32)
        at = {}
        for x in w:
            at[int(x) & CH32_IDX_MASK] = int(x) >> CH32_LEN_SHIFT
        out = []
        for i in range(len(keys)):
            if not counted[i]:
                continue
            k = int(keys[i])
            ring = self.rings.get(k)
            if ring is None:
                ring = self.rings[k] = deque(maxlen=self.M)
            L = at.get(i)
            if L is not None:
                if L > len(ring):
                    raise EvictedRow(f"CHAIN32 word names {L} events before batch row {i}; key {k} holds {len(ring)}")
                chain = list(ring)[len(ring) - L:] if L else []
                out.append((i, [chain, [seq0 + i]]))
            ring.append(seq0 + i)
        return out
