#!/usr/bin/env python3
"""Experiment: the same RMAT graph with vertex ids relabelled in degree order
(highest degree = id 0) against the generator's scrambled ids -- same roots
(translated), per-level device times.  Answers whether degree-ordered ids
(probe locality) are worth building into the engine."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_cuda_bfs_amd as dbfs  # noqa: E402
from distributed_cuda_bfs_amd.parallel.runtime import init_runtime  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
p = dbfs.rmat_params(scale, 16, 1)
t = time.time()
u, v = (np.asarray(x) for x in dbfs.generate_edges(p))
print(f"edges {len(u)} in {time.time() - t:.1f}s", flush=True)
deg = np.bincount(u, minlength=p.n) + np.bincount(v, minlength=p.n)
order = np.lexsort((np.arange(p.n), -deg))       # highest degree first, ties by id
perm = np.empty(p.n, dtype=np.uint32)
perm[order] = np.arange(p.n, dtype=np.uint32)   # old id -> new id
rt = init_runtime("hip")
a = dbfs.BFS(dbfs.build_csr(p.n, u, v), rt)
t = time.time()
b = dbfs.BFS(dbfs.build_csr(p.n, perm[u], perm[v]), rt)
print(f"relabelled graph built in {time.time() - t:.1f}s", flush=True)
roots = a.sample_roots(12, seed=5)
ta = tb = 0.0
for r in roots:
    a.run(r); b.run(int(perm[r]))
    ra, rb = a.run(r), b.run(int(perm[r]))
    assert ra.edges == rb.edges and ra.depth == rb.depth
    ta += ra.ms
    tb += rb.ms
    print(r, f"{ra.ms:.3f} -> {rb.ms:.3f} ms", "".join(l["dir"] for l in ra.levels), "".join(l["dir"] for l in rb.levels),
          [round(l["ms"] * 1e3, 1) for l in ra.levels], [round(l["ms"] * 1e3, 1) for l in rb.levels], flush=True)
print(f"mean {ta / len(roots):.3f} -> {tb / len(roots):.3f} ms per BFS")
