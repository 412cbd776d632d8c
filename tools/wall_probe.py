#!/usr/bin/env python3
"""Where a back-to-back traversal's wall time goes (one GPU, RMAT-26 by default):
run_many over the bench's roots, then per traversal the engine's own time
(res.ms: first enqueue to the host seeing the last stamp), the device-clock
level times and gaps inside it, and the wall time between traversals.

  python3 tools/wall_probe.py [--scale 26] [--roots 16] [--reps 3]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_cuda_bfs_amd as dbfs  # noqa: E402
from distributed_cuda_bfs_amd.parallel.runtime import init_runtime  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=26)
ap.add_argument("--roots", type=int, default=16)
ap.add_argument("--seed", type=int, default=2)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--opt", action="append", default=[])
args = ap.parse_args()
rt = init_runtime("hip")
bfs = dbfs.BFS(dbfs.rmat_params(args.scale, 16, 1), rt, mode="do")
for kv in args.opt:
    k, _, v = kv.partition("=")
    bfs.engine.set_option(k, float(v))
roots = bfs.sample_roots(args.roots, seed=args.seed)
bfs.run_many(roots[:4])
for rep in range(args.reps):
    rt.backend.synchronize()
    t0 = time.perf_counter()
    res = bfs.run_many(roots)
    rt.backend.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    eng = sum(r.ms for r in res)
    dev = sum(sum(lv["ms"] for lv in r.levels) for r in res)
    gaps = sum(sum(max(lv.get("gap_ms", 0.0), 0.0) for lv in r.levels) for r in res)
    n = len(res)
    print(f"rep {rep}: wall {wall / n * 1e3:.1f} us per traversal; engine {eng / n * 1e3:.1f}; device levels "
          f"{dev / n * 1e3:.1f}; gaps between levels {gaps / n * 1e3:.1f}; engine - levels - gaps "
          f"{(eng - dev - gaps) / n * 1e3:.1f}; wall - engine {(wall - eng) / n * 1e3:.1f}; "
          f"GTEPS {sum(r.edges for r in res) / (wall * 1e6):.1f}", flush=True)
