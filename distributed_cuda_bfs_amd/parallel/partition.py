"""1D block vertex partition (owner-computes).

Reference: ``getDev`` / ``v / part`` with ``part = N / P`` (bfs.cu:29-32,148,585),
which maps the tail of ``N % P != 0`` to a non-existent owner.  Here ``part`` is
``ceil(N / P)`` rounded up to 64 vertices so every rank's bitmap slice is a whole
number of 64-bit words and the per-level exchange uses equal-size collectives.
"""
from __future__ import annotations

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

    def __repr__(self) -> str:
        return f"Partition(n={self.n}, nranks={self.nranks}, part={self.part})"
