#!/usr/bin/env python3
"""Traverse chosen roots of the headline RMAT graph (for kernel traces of one
root's levels):  python3 tools/run_roots.py --scale 26 --roots 31811289 40169219
[--opt NAME=VALUE ...].  Each root runs twice (warm-up, then the traced run)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_cuda_bfs_amd as dbfs  # noqa: E402
from distributed_cuda_bfs_amd.parallel.runtime import init_runtime  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=26)
ap.add_argument("--edge-factor", type=int, default=16)
ap.add_argument("--mode", default="do")
ap.add_argument("--roots", type=int, nargs="+", required=True)
ap.add_argument("--opt", action="append", default=[])
args = ap.parse_args()
rt = init_runtime("hip")
bfs = dbfs.BFS(dbfs.rmat_params(args.scale, args.edge_factor, 1), rt, mode=args.mode)
for kv in args.opt:
    k, _, v = kv.partition("=")
    bfs.engine.set_option(k, float(v))
for r in args.roots:
    bfs.run(r)
    res = bfs.run(r)
    print(r, f"{res.ms:.3f} ms", "".join(lv["dir"] for lv in res.levels),
          [lv["frontier_edges"] for lv in res.levels], [round(lv["ms"] * 1e3, 1) for lv in res.levels],
          f"mispredicts {res.mispredicts}", "chains " + " ".join(f"{L}{f}" for L, f, *_ in res.chains),
          "gap-us", [round(lv.get("gap_ms", -1.0) * 1e3, 1) for lv in res.levels],
          f"unaccounted {res.ms * 1e3 - sum(lv['ms'] for lv in res.levels) * 1e3:.1f} us", flush=True)
