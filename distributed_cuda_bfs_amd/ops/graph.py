"""Graph construction, synthetic generators and the CPU oracle.

Reference counterparts: ``readGraphFromFile`` (bfs.cu:829-880, edge list only),
the dead random generator ``readGraph`` (bfs.cu:882-920) and the sequential
oracle ``bfsCPU`` (bfs.cu:923-945).  All heavy lifting is native C++.
"""
from __future__ import annotations

import numpy as np

from .._native import N


def read_graph(path: str, verbose: bool = False, directed: bool = False):
    """Edge list (``n m`` + ``u v`` lines), MatrixMarket (.mtx) or binary CSR -> HostCSR
    (``"-"`` reads standard input).  ``directed`` keeps the pairs as u -> v edges (the
    reference's stdin reader ``readGraph``, bfs.cu:882-920) instead of symmetrising."""
    return N.read_graph(path, verbose, directed)


def read_edge_list(path: str):
    """Return ``(n, u, v)`` numpy arrays of the undirected input edges."""
    return N.read_edge_list(path)


def detect_format(path: str) -> str:
    return N.detect_format(path)


def build_csr(n: int, u, v, directed: bool = False):
    """CSR in the reference's adjacency order (dups and self-loops kept), symmetrised unless directed."""
    return N.build_csr(int(n), np.ascontiguousarray(u, dtype=np.uint32), np.ascontiguousarray(v, dtype=np.uint32),
                       bool(directed))


def rmat_params(scale: int, edge_factor: int = 16, seed: int = 1, scramble: bool = True):
    p = N.rmat_params(int(scale), int(edge_factor), int(seed))
    p.scramble = bool(scramble)
    return p


def uniform_params(n: int, m: int, seed: int = 1):
    return N.uniform_params(int(n), int(m), int(seed))


def power_law_params(n: int, m: int, dmax: int, seed: int = 1):
    """Chung-Lu power-law graph (degree tail exponent 2.5) of n vertices and m
    input edges whose largest expected degree is about dmax -- generated on
    the device like RMAT (rmat.hpp).  The soc-LiveJournal1 / Friendster
    stand-ins: LJ_SIZED_POWER_LAW, FRIENDSTER_SIZED_POWER_LAW."""
    return N.power_law_params(int(n), int(m), int(dmax), int(seed))


def grid_params(w: int, h: int):
    """The w x h grid graph (each vertex joined to its right and lower
    neighbour; row-major labels): road-like, degree <= 4, diameter w + h - 2
    -- the high-diameter case, where a traversal is thousands of tiny levels
    and the per-level latency is everything.  Generated on the device."""
    return N.grid_params(int(w), int(h))


# soc-LiveJournal1 (SNAP: 4,847,571 V, 68,993,773 E; largest undirected degree
# 20,333) and Friendster (65,608,366 V, 1,806,067,135 E; degrees capped at
# 5,000 friends, largest 5,214): (n, m, dmax) of their power-law stand-ins.
LJ_SIZED_POWER_LAW = (4847571, 68993773, 20333)
FRIENDSTER_SIZED_POWER_LAW = (65608366, 1806067135, 5214)


def generate_edges(params, begin: int = 0, end: int = -1):
    """Host copy of the counter-based edge stream (bit-identical to the device generator)."""
    return N.generate_edges(params, int(begin), int(end))


def host_csr_from_params(params):
    u, v = generate_edges(params)
    return build_csr(params.n, u, v)


def cpu_bfs(csr, src: int):
    """Sequential oracle: returns ``(levels int32, parent_edge int64)``; unreached = INT32_MAX."""
    return N.cpu_bfs(csr, int(src))


def write_binary_csr(path: str, csr) -> None:
    N.write_binary_csr(path, csr)


def write_levels(path: str, levels) -> None:
    N.write_levels(path, np.ascontiguousarray(levels, dtype=np.int32))
