"""Host-side BFS result checks.

``check_levels_against_oracle`` is the reference's ``checkOutput``
(bfs.cu:374-384): element-wise level equality against the CPU oracle, reporting
the first mismatch.  ``levels_are_consistent`` is the Graph500 level test on the
host (the device version is ``Engine.validate``).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

UNREACHED = np.iinfo(np.int32).max


def check_levels_against_oracle(got, expected) -> Optional[Tuple[int, int, int]]:
    got = np.asarray(got)
    expected = np.asarray(expected)
    if got.shape != expected.shape:
        return (-1, int(got.size), int(expected.size))
    bad = np.nonzero(got != expected)[0]
    if bad.size == 0:
        return None
    i = int(bad[0])
    return (i, int(got[i]), int(expected[i]))


def levels_are_consistent(csr, levels, src: int) -> bool:
    lv = np.asarray(levels, dtype=np.int64)
    ro = np.asarray(csr.row_off)
    col = np.asarray(csr.col)
    if lv[src] != 0:
        return False
    rows = np.repeat(np.arange(csr.n), np.diff(ro))
    lu, lw = lv[rows], lv[col]
    ru, rw = lu != UNREACHED, lw != UNREACHED
    if np.any(ru != rw):
        return False
    both = ru & rw
    if np.any(np.abs(lu[both] - lw[both]) > 1):
        return False
    has_parent = np.zeros(csr.n, dtype=bool)
    m = both & (lw == lu - 1)
    has_parent[rows[m]] = True
    reached = lv != UNREACHED
    reached[src] = False
    return bool(np.all(has_parent[reached]))


def parents_are_valid(csr, levels, parents, src: int) -> bool:
    """Graph500 parent-tree check: every reached v != src has an edge to
    parent[v] and level[parent[v]] == level[v] - 1; unreached have -1."""
    lv = np.asarray(levels, dtype=np.int64)
    par = np.asarray(parents, dtype=np.int64)
    ro = np.asarray(csr.row_off)
    col = np.asarray(csr.col)
    if par[src] != src:
        return False
    for v in range(csr.n):
        if v == src:
            continue
        if lv[v] == UNREACHED:
            if par[v] != -1:
                return False
            continue
        p = par[v]
        if p < 0 or lv[p] != lv[v] - 1:
            return False
        if p not in col[ro[v]:ro[v + 1]]:
            return False
    return True
