"""Graph operations backed by the native core (I/O, CSR build, generators, oracle)."""
from .graph import (  # noqa: F401
    read_graph, read_edge_list, build_csr, rmat_params, uniform_params, power_law_params, grid_params, generate_edges,
    host_csr_from_params, cpu_bfs, write_binary_csr, write_levels, detect_format)
