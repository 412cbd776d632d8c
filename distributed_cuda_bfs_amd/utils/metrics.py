"""Graph500 traversal metrics.

TEPS = traversed undirected input edges (sum of degrees over reached vertices
/ 2) / BFS time.  The reference computes no TEPS at all; it prints the level
loop's wall time in whole milliseconds (bfs.cu:551,624-626).
"""
from __future__ import annotations

from typing import Iterable, List, Sequence


def gteps(edges: int, ms: float) -> float:
    return edges / (ms * 1e6) if ms > 0 else 0.0


def harmonic_mean(xs: Iterable[float]) -> float:
    xs = [x for x in xs]
    if not xs or any(x <= 0 for x in xs):
        return 0.0
    return len(xs) / sum(1.0 / x for x in xs)


def summarize_runs(results: Sequence) -> dict:
    ms = [r.ms for r in results]
    ge = [r.gteps for r in results]
    edges = sum(r.edges for r in results)
    tot = sum(ms)
    srt: List[float] = sorted(ms)
    return {
        "runs": len(results),
        "mean_ms": tot / len(ms) if ms else 0.0,
        "median_ms": srt[len(srt) // 2] if srt else 0.0,
        "min_ms": srt[0] if srt else 0.0,
        "max_ms": srt[-1] if srt else 0.0,
        "aggregate_gteps": gteps(edges, tot),
        "harmonic_mean_gteps": harmonic_mean(ge),
    }
