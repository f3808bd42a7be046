"""TEST INFRASTRUCTURE ONLY -- restatement of the reference's chained-bucket voxel hash.

Follows hash_fusion.py:199-437 and data_structures/bucket.py:9-131 operation by operation
(5-slot buckets, the last slot's entry heads an overflow chain of (bucket, slot) offsets,
linear probe for the next bucket with a free slot among 0..3, resize by doubling when
non-empty/n >= 0.75 BEFORE an insert, no de-duplication).  Storage is flat arrays instead of
Python objects so that the author's recorded counts can be replayed in seconds:

  * Bucket.__init__ calls  == `buckets_created`
  * _add_to_linked_list calls == `overflows`

(298,500 / 0 for lounge frame 0 and 322,698 / 4 for frames 0-9, int32 keys.)
"""
from __future__ import annotations

import numpy as np

P1, P2, P3 = 73856093, 19349669, 83492791
BUCKET = 5


def hash_value(pos, n: int, int_bits: int = 64) -> int:
    """hash_fusion.py:182-190 for one coordinate triple."""
    x, y, z = (int(v) for v in pos)
    if int_bits == 32:
        def w(a):
            a &= 0xFFFFFFFF
            return a - (1 << 32) if a >= (1 << 31) else a
        h = w(w(x * P1) ^ w(y * P2) ^ w(z * P3))
    else:
        def w(a):
            a &= 0xFFFFFFFFFFFFFFFF
            return a - (1 << 64) if a >= (1 << 63) else a
        h = w(w(x * P1) ^ w(y * P2) ^ w(z * P3))
    return h % n  # Python % == np.remainder (sign of divisor)


class BucketTable:
    def __init__(self, n: int, int_bits: int = 64, load_factor: float = 0.75):
        self.n = int(n)
        self.int_bits = int_bits
        self.load_factor = load_factor
        self.slots = np.full((self.n, BUCKET), -1, np.int64)  # entry id or -1
        self.alive = np.zeros(self.n, bool)  # bucket object exists (not None)
        self.nonempty = 0
        self.pos: list = []      # entry id -> position tuple
        self.off: list = []      # entry id -> (bucket, slot) or None
        self.buckets_created = 0
        self.overflows = 0
        self.resizes = 0

    # -- helpers -------------------------------------------------------------------------
    def _h(self, pos):
        return hash_value(pos, self.n, self.int_bits)

    def _new_bucket(self, b, eid):
        self.slots[b, :] = -1
        self.slots[b, 0] = eid
        self.alive[b] = True
        self.nonempty += 1
        self.buckets_created += 1

    # -- hash_fusion.py:199-224 -----------------------------------------------------------
    def add(self, pos):
        pos = tuple(int(v) for v in pos)
        eid = len(self.pos)
        self.pos.append(pos)
        self.off.append(None)
        return self._add_eid(eid)

    def _add_eid(self, eid):
        if self.nonempty / self.n >= self.load_factor:
            self.double_table_size()
        h = self._h(self.pos[eid])
        if not self.alive[h]:
            self._new_bucket(h, eid)
            return h, 0
        row = self.slots[h]
        free = np.flatnonzero(row < 0)
        if free.size == 0:
            return self._add_to_linked_list(h, eid)
        row[free[0]] = eid
        return h, int(free[0])

    # -- hash_fusion.py:226-276 -----------------------------------------------------------
    def _add_to_linked_list(self, h, eid):
        self.overflows += 1
        last = int(self.slots[h, BUCKET - 1])
        b, s = h, BUCKET - 1
        while self.off[last] is not None:
            b, s = self.off[last]
            last = int(self.slots[b, s])
        return self._find_next_free(b, s, last, eid)

    def _find_next_free(self, begin_b, begin_e, prev, eid):
        b = begin_b
        if begin_e < BUCKET - 1:
            row = self.slots[b]
            for i in range(begin_e, BUCKET - 1):
                if row[i] < 0:
                    row[i] = eid
                    self.off[prev] = (begin_b, i)
                    return begin_b, i
        while True:
            b = 0 if b >= self.n - 1 else b + 1
            if not self.alive[b]:
                self._new_bucket(b, eid)
                self.off[prev] = (b, 0)
                return b, 0
            row = self.slots[b]
            if (row[:BUCKET - 1] >= 0).all():
                if b == begin_b:
                    return -1, -1
            else:
                i = int(np.flatnonzero(row < 0)[0])
                row[i] = eid
                self.off[prev] = (b, i)
                return b, i

    # -- hash_fusion.py:285-310 -----------------------------------------------------------
    def get(self, pos):
        pos = tuple(int(v) for v in pos)
        h = self._h(pos)
        if not self.alive[h]:
            return None
        row = self.slots[h]
        if (row < 0).all():
            return None
        for e in row:
            if e >= 0 and self.pos[e] == pos:
                return int(e)
        last = int(row[BUCKET - 1])
        if last >= 0 and self.off[last] is not None:
            b, s = self.off[last]
            nxt = int(self.slots[b, s])
            while True:
                if self.pos[nxt] == pos:
                    return nxt
                if self.off[nxt] is None:
                    break
                b, s = self.off[nxt]
                nxt = int(self.slots[b, s])
        return None

    # -- hash_fusion.py:330-393 -----------------------------------------------------------
    def _remove_at(self, b, s):
        if self.alive[b]:
            self.slots[b, s] = -1
            if (self.slots[b] < 0).all():
                self.alive[b] = False
                self.nonempty -= 1

    def remove(self, pos):
        pos = tuple(int(v) for v in pos)
        h = self._h(pos)
        if not self.alive[h] or (self.slots[h] < 0).all():
            return 0
        row = self.slots[h]
        last = None
        for i in range(BUCKET):
            e = int(row[i])
            if e < 0:
                continue
            last = e
            if self.pos[e] == pos:
                if self.off[e] is None:
                    row[i] = -1
                    if (row < 0).all():
                        self.alive[h] = False
                        self.nonempty -= 1
                    return 1
                b, s = self.off[e]
                nxt = int(self.slots[b, s])
                self._remove_at(b, s)
                row[i] = nxt
                return 1
        if last is not None:
            cur = last
            while self.off[cur] is not None:
                b, s = self.off[cur]
                nxt = int(self.slots[b, s])
                if self.pos[nxt] == pos:
                    self.off[cur] = self.off[nxt]
                    self._remove_at(b, s)
                    return 1
                cur = nxt
        return 0

    # -- hash_fusion.py:414-437 -----------------------------------------------------------
    def double_table_size(self):
        self.resizes += 1
        old_slots, old_alive = self.slots, self.alive
        self.n *= 2
        self.slots = np.full((self.n, BUCKET), -1, np.int64)
        self.alive = np.zeros(self.n, bool)
        self.nonempty = 0
        for b in np.flatnonzero(old_alive):
            for e in old_slots[b]:
                if e >= 0:
                    self.off[int(e)] = None
                    self._add_eid(int(e))

    # -- hash_fusion.py:147-180 -----------------------------------------------------------
    def count_entries(self) -> int:
        return int((self.slots[self.alive] >= 0).sum())

    def load_factor_now(self) -> float:
        return self.nonempty / self.n

    def collisions(self) -> int:
        return int(((self.slots[self.alive] >= 0).sum(1) > 1).sum())
