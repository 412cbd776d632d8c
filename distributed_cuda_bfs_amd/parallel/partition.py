"""1D block vertex partition (owner-computes).

Reference: ``getDev`` / ``v / part`` with ``part = N / P`` (bfs.cu:29-32,148,585),
which maps the tail of ``N % P != 0`` to a non-existent owner.  Here ``part`` is
``ceil(N / P)`` rounded up to 64 vertices so every rank's bitmap slice is a whole
number of 64-bit words and the per-level exchange uses equal-size collectives.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from .._native import N


class Partition:
    def __init__(self, n: int, nranks: int):
        self._p = N.Partition(int(n), int(nranks))

    @property
    def native(self):
        return self._p

    @property
    def n(self) -> int:
        return self._p.n

    @property
    def nranks(self) -> int:
        return self._p.nranks

    @property
    def part(self) -> int:
        return self._p.part

    def owner(self, v: int) -> int:
        return self._p.owner(int(v))

    def lo(self, r: int) -> int:
        return self._p.lo(int(r))

    def hi(self, r: int) -> int:
        return self._p.hi(int(r))

    def count(self, r: int) -> int:
        return self._p.count(int(r))

    def slice_words(self) -> int:
        return self._p.slice_words()

    # ---- vectorised (numpy) forms: owner routing of whole vertex arrays ----
    # The native Partition answers one vertex at a time; these work on arrays
    # (host-side routing of edge lists or frontiers, result assembly, tests).

    def owners(self, v) -> np.ndarray:
        """Owner rank of every vertex id in ``v`` (int32 array)."""
        v = np.asarray(v, dtype=np.int64)
        if v.size and (v.min() < 0 or v.max() >= self.n):
            raise ValueError("vertex id out of range [0, n)")
        return np.minimum(v // self.part, self.nranks - 1).astype(np.int32)

    def to_local(self, v) -> np.ndarray:
        """Local row of every vertex on its owner (v - lo(owner(v)))."""
        v = np.asarray(v, dtype=np.int64)
        return v - self.owners(v).astype(np.int64) * self.part

    def to_global(self, r: int, local) -> np.ndarray:
        """Global ids of rank r's local rows ``local``."""
        local = np.asarray(local, dtype=np.int64)
        if local.size and (local.min() < 0 or local.max() >= self.count(r)):
            raise ValueError(f"local row out of range for rank {r}")
        return local + self.lo(r)

    def route(self, v) -> List[np.ndarray]:
        """Owner buckets: ``out[r]`` = the entries of ``v`` owned by rank r, in
        input order (what the reference's per-owner queues hold, bfs.cu:148-150;
        the engine does this on the device with wave-aggregated appends)."""
        v = np.asarray(v, dtype=np.int64)
        own = self.owners(v)
        order = np.argsort(own, kind="stable")
        bounds = np.searchsorted(own[order], np.arange(self.nranks + 1))
        return [v[order[bounds[r]:bounds[r + 1]]] for r in range(self.nranks)]

    def split(self, per_vertex) -> List[np.ndarray]:
        """A length-n per-vertex array cut into the ranks' owned slices."""
        a = np.asarray(per_vertex)
        if a.shape[0] != self.n:
            raise ValueError("per-vertex array must have n entries")
        return [a[self.lo(r):self.hi(r)] for r in range(self.nranks)]

    def assemble(self, slices: Sequence) -> np.ndarray:
        """Inverse of split: the ranks' owned slices concatenated in rank order
        (what the engine's level all-gather produces)."""
        if len(slices) != self.nranks:
            raise ValueError("one slice per rank")
        for r, sl in enumerate(slices):
            if len(sl) != self.count(r):
                raise ValueError(f"slice {r} has {len(sl)} entries, rank owns {self.count(r)}")
        return np.concatenate([np.asarray(sl) for sl in slices]) if self.nranks else np.empty(0)

    def __repr__(self) -> str:
        return f"Partition(n={self.n}, nranks={self.nranks}, part={self.part})"
