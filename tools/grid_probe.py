#!/usr/bin/env python3
"""High-diameter probe: the W x H grid on one GPU, per-level device-clock
time and the idle gap before each level (the per-level fixed cost).

  python tools/grid_probe.py --grid 1024:1024 --roots 0 524800 --mode td
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", default="1024:1024")
    ap.add_argument("--roots", type=int, nargs="+", default=[0, 524800])
    ap.add_argument("--mode", default="td")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE")
    args = ap.parse_args()
    import numpy as np

    import distributed_cuda_bfs_amd as dbfs
    from distributed_cuda_bfs_amd.parallel.runtime import init_runtime

    w, _, h = args.grid.partition(":")
    p = dbfs.grid_params(int(w), int(h))
    rt = init_runtime("auto")
    b = dbfs.BFS(p, rt, mode=args.mode)
    for kv in args.opt:
        k, _, v = kv.partition("=")
        b.engine.set_option(k, float(v))
    b.run(args.roots[0])  # (warm-up; a deep traversal also settles the level width)
    for r in args.roots:
        for _ in range(args.reps):
            t0 = time.perf_counter()
            res = b.run(r)
            wall = (time.perf_counter() - t0) * 1e3
        lv = res.levels
        ms = np.array([x["ms"] for x in lv])
        gap = np.array([max(x.get("gap_ms", 0.0), 0.0) for x in lv])
        forms = "".join(c[1] for c in res.chains)
        print(f"root {r}: depth {res.depth}, {res.ms:.3f} ms ({wall:.3f} ms wall), "
              f"{1e3 * res.ms / res.depth:.2f} us/level; device level {1e3 * ms.mean():.2f} us "
              f"(median {1e3 * np.median(ms):.2f}), gap {1e3 * gap.mean():.2f} us; chains {len(res.chains)} "
              f"({forms[:12]}...), mispredicts {res.mispredicts}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
