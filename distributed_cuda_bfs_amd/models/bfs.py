"""High-level distributed BFS.

Reference entry points: ``main`` -> ``runCudaQueueBfs`` (bfs.cu:783-823,
542-629) and the MPI variant (bfs_mpi.cu:797-856).  One ``BFS`` object holds
this rank's CSR shard on its device and a native engine; ``run(src)`` is one
level-synchronous traversal (all ranks call it collectively).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Union

import numpy as np

from .._native import N
from ..parallel.runtime import Runtime, init_runtime

MODES = ("ref", "td", "bu", "do", "simple", "scan")


class BFSResult:
    """One traversal: totals, plus per-level records (list of dicts with level,
    dir, frontier, frontier_edges, discovered, ms, comm_ms, gap_ms) converted
    from the native record on first access."""

    __slots__ = ("source", "ms", "reached", "edges", "depth", "gteps", "mispredicts", "_native", "_levels")

    def __init__(self, source: int, ms: float, reached: int, edges: int, depth: int, gteps: float,
                 levels: Optional[List[Dict[str, Any]]] = None, mispredicts: int = 0, native: Any = None):
        self.source, self.ms, self.reached, self.edges = source, ms, reached, edges
        self.depth, self.gteps, self.mispredicts = depth, gteps, mispredicts
        self._native, self._levels = native, levels

    @property
    def chains(self) -> List[Any]:
        """Device loop: every level chain enqueued, in order, as (level, form,
        list capacity, gathered, pushed, unvisited filter, parts)
        -- form T / S / L / B / X (mispredicted chains included); parts > 1: a
        split top-down level (Options td_split_edges / td_split_parts)."""
        return list(self._native.chains) if self._native is not None else []

    @property
    def levels(self) -> List[Dict[str, Any]]:
        if self._levels is None:
            self._levels = list(self._native.level_dicts()) if self._native is not None else []
        return self._levels

    def __repr__(self) -> str:
        return (f"BFSResult(source={self.source}, ms={self.ms:.4f}, reached={self.reached}, edges={self.edges}, "
                f"depth={self.depth}, gteps={self.gteps:.2f})")

    @classmethod
    def from_native(cls, r: Any) -> "BFSResult":
        if isinstance(r, dict):
            return cls(r["source"], r["ms"], r["reached"], r["edges"], r["depth"], r["gteps"],
                       levels=list(r["levels"]), mispredicts=int(r.get("mispredicts", 0)))
        return cls(r.source, r.ms, r.reached, r.edges, r.depth, r.gteps, mispredicts=r.mispredicts, native=r)


class BFS:
    """Distributed BFS over a graph given as a HostCSR, generator params, or a file path."""

    def __init__(self, graph: Union[str, Any], runtime: Optional[Runtime] = None, mode: str = "do",
                 alpha: float = 40.0, beta: float = 384.0, bu_lane_limit: int = 16, phase_timing: bool = False,
                 hub_sort: bool = True, force_exchange: bool = False, hubs: bool = True,
                 max_hubs: Optional[int] = None, directed: bool = False, sharded: bool = True,
                 read_threads: int = 0, id_order: bool = True):
        """``hub_sort`` reorders every adjacency row by neighbour degree (descending)
        once, before any traversal: levels are unchanged, bottom-up probes find a
        frontier parent sooner (see csrc/kernels/graph_sort.hip).  ``hubs`` also
        indexes the highest-degree vertices so that bottom-up probes of them test
        an LDS-resident copy of their frontier bits (needs ``hub_sort``); with
        hubs and ``id_order`` the top-down copy of the adjacency is then put in
        neighbour-id order (bottom-up keeps the hub-first order).

        A file path is read in shards (``sharded``, the default for undirected
        files): every rank parses only its byte range of an edge list /
        MatrixMarket file with ``read_threads`` host threads and the CSR shard
        is built on its GPU (edges routed to their owners by an all-to-all-v),
        or reads only its rows of a binary CSR cache.  ``sharded=False`` reads
        the whole file on every rank (the reference's bfs_mpi.cu:815 pattern)."""
        if mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}")
        self.rt = runtime or init_runtime()
        if directed and mode in ("bu", "do"):
            raise ValueError("directed graphs need a top-down mode (td, ref, simple, scan)")
        if isinstance(graph, str) and not (sharded and not directed and graph != "-"):
            graph = N.read_graph(graph, False, directed)
        if isinstance(graph, str):
            self.graph = N.DeviceGraph.from_file(self.rt.backend, self.rt.comm, graph, int(read_threads))
            self.n = self.graph.n
            self.partition = self.graph.partition
        elif isinstance(graph, N.GenParams):
            self.n = graph.n
            self.partition = N.Partition(graph.n, self.rt.world)
            self.graph = N.DeviceGraph.generate(self.rt.backend, graph, self.partition, self.rt.rank)
        elif isinstance(graph, N.HostCSR):
            self.n = graph.n
            self.partition = N.Partition(graph.n, self.rt.world)
            self.graph = N.DeviceGraph.from_host(self.rt.backend, graph, self.partition, self.rt.rank)
        else:
            raise TypeError("graph must be a path, HostCSR or GenParams")
        if hub_sort:
            cap = N.MAX_HUBS if max_hubs is None else int(max_hubs)
            self.graph.sort_neighbors_by_degree(self.rt.comm, hubs, cap, id_order)
        self.engine = N.Engine(self.graph, self.rt.comm, mode=mode, alpha=alpha, beta=beta,
                               bu_lane_limit=bu_lane_limit, phase_timing=phase_timing,
                               force_exchange=force_exchange)
        if directed:  # the CSR holds out-edges only (see build_csr / read_graph)
            self.engine.set_option("directed", 1)

    def use_comm(self, comm) -> None:
        """Rebuild the engine on another communicator (same shard, same
        options): e.g. the RCCL communicator a peer-memory one wraps."""
        opts = dict(self.engine.get_options())
        mode = self.engine.mode
        self.rt.comm = comm
        comm.bind_backend(self.rt.backend)
        self.engine = N.Engine(self.graph, comm, mode=mode, alpha=opts["alpha"], beta=opts["beta"],
                               bu_lane_limit=int(opts["bu_lane_limit"]), phase_timing=bool(opts["phase_timing"]),
                               force_exchange=bool(opts["force_exchange"]))
        for k, v in opts.items():
            self.engine.set_option(k, v)

    @property
    def mode(self) -> str:
        return self.engine.mode

    @mode.setter
    def mode(self, m: str) -> None:
        if m not in MODES:
            raise ValueError(f"mode must be one of {MODES}")
        self.engine.mode = m

    def run(self, source: int) -> BFSResult:
        return BFSResult.from_native(self.engine.run(int(source)))

    def run_many(self, sources) -> List[BFSResult]:
        """One complete traversal per source, back to back in native code (no
        return to Python between them: the host gap between two traversals is
        the engine's own).  Collective like run()."""
        return [BFSResult.from_native(r) for r in self.engine.run_many([int(s) for s in sources])]

    def levels(self) -> np.ndarray:
        """Full per-vertex level array of the last run (collective)."""
        return self.engine.gather_levels()

    def local_levels(self) -> np.ndarray:
        return self.engine.levels_local()

    def parents(self, source: int) -> np.ndarray:
        """Graph500 parent tree of the last run from ``source`` (collective).

        parent[v] is a neighbour one level closer to the source (global vertex
        id), parent[source] = source, -1 for unreached vertices.  The reference
        records edge indices as parents and never gathers them (bfs.cu:147,439).
        """
        return self.engine.gather_parents(int(source))

    def validate(self, source: int) -> bool:
        """Graph500-style level validation of the last run on the device (collective)."""
        gap, cross, orphan = self.engine.validate(int(source))
        return gap == 0 and cross == 0 and orphan == 0

    def degree(self, v: int) -> int:
        """Degree of global vertex v (collective: the owner contributes)."""
        own = self.partition.owner(int(v))
        d = 0
        if own == self.rt.rank:
            d = self.graph.degrees_of([int(v) - self.partition.lo(own)])[0]
        return int(self.rt.comm.sum_host(int(d))) if self.rt.world > 1 else int(d)

    def sample_roots(self, k: int, seed: int = 1) -> List[int]:
        """Graph500 root sampling: k distinct random vertices of degree >= 1 (collective)."""
        rng = np.random.default_rng(seed)
        roots: List[int] = []
        seen = set()
        tries = 0
        while len(roots) < k and tries < 64 * k + 64:
            tries += 1
            v = int(rng.integers(0, self.n))
            if v in seen:
                continue
            seen.add(v)
            if self.degree(v) > 0:
                roots.append(v)
        return roots
