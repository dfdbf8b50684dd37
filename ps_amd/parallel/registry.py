"""Key registry and range partitioner.

The reference addresses parameters by string key and shards keys over servers with
``key.hashCode() % n`` (net/Mod.java:14, net/PSRouterClient.java:44-58) -- which crashes for
negative hash codes (Q4) and balances bytes poorly.  Here every dense key is placed in a
flat per-dtype buffer; the buffer is cut into *buckets* (the unit of communication and of
compute/communication overlap) and every bucket is cut into ``world_size`` equal, aligned
*chunks*: rank r owns chunk r of every bucket.  Ownership is therefore a contiguous range
per bucket ("range partition"), perfectly byte-balanced, and a push of a bucket is exactly
one reduce-scatter, a pull exactly one all-gather.

Keys are registered in the order gradients become ready during backward (reverse of the
forward order), so bucket 0 is ready first.  The final bucket (holding the first layers,
ready last, needed first by the next forward) is capped small to shrink the exposed tail.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch


@dataclass
class KeyInfo:
    name: str
    shape: Tuple[int, ...]
    numel: int
    dtype: torch.dtype
    group: str
    bucket: int = -1
    offset: int = -1  # element offset inside the group buffer


@dataclass
class Bucket:
    index: int
    group: str
    start: int  # element offset inside the group buffer
    size: int  # padded element count (multiple of world * align)
    world: int
    keys: List[str] = field(default_factory=list)

    @property
    def chunk(self) -> int:
        return self.size // self.world

    def owner_range(self, rank: int) -> Tuple[int, int]:
        """[lo, hi) element range of ``rank``'s chunk inside the group buffer."""
        lo = self.start + rank * self.chunk
        return lo, lo + self.chunk


def _gname(dt: torch.dtype) -> str:
    return str(dt).replace("torch.", "")


class Registry:
    def __init__(self, world_size: int = 1, bucket_bytes: int = 32 << 20, align: int = 64,
                 last_bucket_bytes: Optional[int] = 4 << 20):
        if world_size < 1:
            raise ValueError("world_size must be >= 1")
        self.world = world_size
        self.bucket_bytes = int(bucket_bytes)
        self.align = int(align)
        self.last_bucket_bytes = last_bucket_bytes
        self.keys: Dict[str, KeyInfo] = {}
        self.order: List[str] = []
        self.buckets: List[Bucket] = []
        self.group_size: Dict[str, int] = {}
        self.group_dtype: Dict[str, torch.dtype] = {}
        self._final = False

    def add(self, name: str, shape: Sequence[int], dtype: torch.dtype) -> KeyInfo:
        if self._final:
            raise RuntimeError("registry already finalized")
        if name in self.keys:
            raise KeyError(f"duplicate key {name!r}")
        shape = tuple(int(s) for s in shape)
        n = 1
        for s in shape:
            n *= s
        ki = KeyInfo(name, shape, n, dtype, _gname(dtype))
        self.keys[name] = ki
        self.order.append(name)
        self.group_dtype[ki.group] = dtype
        return ki

    def finalize(self) -> "Registry":
        """Assign keys to buckets (greedy, in registration order) and compute offsets."""
        quantum = self.world * self.align
        by_group: Dict[str, List[str]] = {}
        for k in self.order:
            by_group.setdefault(self.keys[k].group, []).append(k)
        for g, names in by_group.items():
            esize = torch.empty((), dtype=self.group_dtype[g]).element_size()
            cap = max(1, self.bucket_bytes // esize)
            # split the key list into buckets of <= cap elements (a key larger than cap gets its own)
            groups: List[List[str]] = []
            cur: List[str] = []
            cur_n = 0
            for k in names:
                n = self.keys[k].numel
                if cur and cur_n + n > cap:
                    groups.append(cur)
                    cur, cur_n = [], 0
                cur.append(k)
                cur_n += n
            if cur:
                groups.append(cur)
            # cap the last bucket (first layers of the net): split its tail off
            if self.last_bucket_bytes and len(names) > 1:
                lcap = max(1, self.last_bucket_bytes // esize)
                last = groups[-1]
                tail: List[str] = []
                tn = 0
                while len(last) > 1 and tn + self.keys[last[-1]].numel <= lcap:
                    k = last.pop()
                    tail.insert(0, k)
                    tn += self.keys[k].numel
                if tail and last:
                    groups.append(tail)
                elif tail:
                    groups[-1] = tail
            off = 0
            for names_b in groups:
                b = Bucket(len(self.buckets), g, off, 0, self.world, list(names_b))
                inner = 0
                for k in names_b:
                    ki = self.keys[k]
                    ki.bucket = b.index
                    ki.offset = off + inner
                    inner += ki.numel
                b.size = ((inner + quantum - 1) // quantum) * quantum
                off += b.size
                self.buckets.append(b)
            self.group_size[g] = off
        self._final = True
        return self

    # ------------------------------------------------------------------ queries
    def owner_of(self, key: str) -> List[Tuple[int, int, int]]:
        """[(rank, lo, hi)] pieces of ``key`` (group-buffer element ranges) and their owners."""
        ki = self.keys[key]
        b = self.buckets[ki.bucket]
        out = []
        lo, hi = ki.offset, ki.offset + ki.numel
        for r in range(self.world):
            olo, ohi = b.owner_range(r)
            a, z = max(lo, olo), min(hi, ohi)
            if a < z:
                out.append((r, a, z))
        return out

    def owned_keys(self, rank: int) -> List[str]:
        return [k for k in self.order if any(r == rank for r, _, _ in self.owner_of(k))]

    def segments(self, bucket: int, rank: int) -> List[Tuple[str, int, int]]:
        """Key pieces inside ``rank``'s chunk of ``bucket`` as (key, lo, hi) group offsets."""
        b = self.buckets[bucket]
        olo, ohi = b.owner_range(rank)
        out = []
        for k in b.keys:
            ki = self.keys[k]
            a, z = max(ki.offset, olo), min(ki.offset + ki.numel, ohi)
            if a < z:
                out.append((k, a, z))
        return out

    def summary(self) -> str:
        lines = [f"Registry(world={self.world}, keys={len(self.keys)}, buckets={len(self.buckets)})"]
        for b in self.buckets:
            esize = torch.empty((), dtype=self.group_dtype[b.group]).element_size()
            lines.append(f"  bucket {b.index} [{b.group}] keys={len(b.keys)} size={b.size} "
                         f"({b.size * esize / 2**20:.2f} MiB) chunk={b.chunk}")
        return "\n".join(lines)


def hash_router(n: int):
    """Reference-compatible key router (net/Mod.java) with the negative-hash crash fixed (Q4):
    Python's modulo is non-negative.  Uses a stable FNV-1a hash instead of Java hashCode."""

    def shard(key: str) -> int:
        h = 0xCBF29CE484222325
        for ch in key.encode():
            h ^= ch
            h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
        return h % n

    return shard
