"""MI355X-native distributed breadth-first search.

A from-scratch re-design of xxcclong/Distributed-CUDA-BFS for AMD MI355X
(gfx950 / CDNA4): CSR graphs 1D vertex-partitioned over the GPUs of a node,
hand-written HIP kernels (load-balanced top-down gather, bottom-up parent
search, bitmap frontier update, wave-prefix-sum compaction), direction
optimisation, and an RCCL all-to-all / all-gather frontier exchange over xGMI.

Layout
  models/    BFS front-ends (the engine modes: ref, td, bu, do, simple, scan)
  ops/       graph construction / generation / oracle operations
  parallel/  partitioning, communicators (RCCL, virtual ranks, torch.distributed)
  utils/     file I/O, Graph500 root sampling, GTEPS accounting, validation
"""
from ._native import N as native  # noqa: F401  (fails loudly if the core is not built)
from .models.bfs import BFS, BFSResult, MODES  # noqa: F401
from .ops.graph import (  # noqa: F401
    read_graph, read_edge_list, detect_format, build_csr, rmat_params, uniform_params, power_law_params, grid_params, generate_edges,
    host_csr_from_params, cpu_bfs, write_binary_csr, write_levels)
from .parallel.partition import Partition  # noqa: F401
from .parallel.runtime import Runtime, init_runtime  # noqa: F401

UNREACHED = native.UNREACHED
__version__ = "0.1.0"
