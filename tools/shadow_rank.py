#!/usr/bin/env python3
"""Shadow-rank measurement: per-level kernel time of rank r of a P-GPU
traversal, measured alone on one GPU (distributed_cuda_bfs_amd/parallel/shadow.py).

  python tools/shadow_rank.py --scale 26 --ranks-of 8 --ranks 0 7 --roots 4

Prints, per root, the one-GPU level times (same roots, one rank) next to the
replayed ranks' level times, plus the collectives each replayed traversal
issued and their bytes; --json writes everything.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--grid", default=None, metavar="W:H", help="the road-like W x H grid instead of RMAT")
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--ranks-of", type=int, default=8, help="P: ranks of the recorded job")
    ap.add_argument("--ranks", type=int, nargs="+", default=[0, 7], help="ranks to replay")
    ap.add_argument("--roots", type=int, default=4)
    ap.add_argument("--root-seed", type=int, default=12345)
    ap.add_argument("--root-list", type=int, nargs="+", default=None, help="explicit roots (instead of sampling)")
    ap.add_argument("--mode", default="do")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()

    import distributed_cuda_bfs_amd as dbfs
    from distributed_cuda_bfs_amd.parallel.runtime import init_runtime
    from distributed_cuda_bfs_amd.parallel.shadow import shadow_ranks

    opts = {k: float(v) for k, v in (kv.split("=", 1) for kv in args.opt)}
    if args.grid:
        gw, _, gh = args.grid.partition(":")
        params = dbfs.grid_params(int(gw), int(gh))
    else:
        params = dbfs.rmat_params(args.scale, args.edge_factor, args.seed)
    t0 = time.time()
    # one rank, same roots: the 1-GPU level times (and the root sample)
    rt = init_runtime(args.device)
    one = dbfs.BFS(params, rt, mode=args.mode)
    for k, v in opts.items():
        one.engine.set_option(k, v)
    roots = args.root_list or one.sample_roots(args.roots, seed=args.root_seed)
    one.run(roots[0])
    ref = []
    for r in roots:
        res = one.run(r)
        ref.append([(lv["dir"], lv["ms"], lv["frontier_edges"]) for lv in res.levels])
    del one
    print(f"[shadow] one-rank reference: {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    t0 = time.time()
    runs = shadow_ranks(params, args.ranks_of, args.ranks, roots, mode=args.mode, device=args.device, opts=opts)
    print(f"[shadow] record + replay: {time.time() - t0:.1f} s", file=sys.stderr, flush=True)

    P = args.ranks_of
    gname = f"grid {args.grid}" if args.grid else f"RMAT-{args.scale} ef{args.edge_factor}"
    print(f"{gname}, mode {args.mode}: rank r of P = {P} replayed alone "
          f"(device-clock level times, us; the P = {P} rank also pays one device copy per collective)")
    for i, root in enumerate(roots):
        print(f"\nroot {root}")
        hdr = f"{'lvl':>3} {'dir':>3} {'frontier edges':>15} {'1 GPU':>8}"
        for s in runs:
            hdr += f" {'r' + str(s.rank) + '/' + str(P):>8}"
        print(hdr)
        n = max(len(ref[i]), *(len(s.levels[i]) for s in runs))
        for L in range(n):
            d, ms, mf = ref[i][L] if L < len(ref[i]) else ("-", 0.0, 0)
            line = f"{L:>3} {d:>3} {mf:>15,} {ms * 1e3:>8.1f}"
            for s in runs:
                lv = s.levels[i]
                line += f" {lv[L][1] * 1e3:>8.1f}" if L < len(lv) else f" {'-':>8}"
            print(line)
        tot = f"{'sum':>3} {'':>3} {'':>15} {sum(x[1] for x in ref[i]) * 1e3:>8.1f}"
        for s in runs:
            tot += f" {sum(x[1] for x in s.levels[i]) * 1e3:>8.1f}"
        print(tot)
        per = f"{'per':>3} {'lvl':>3} {'(us per level)':>15} {sum(x[1] for x in ref[i]) * 1e3 / max(len(ref[i]), 1):>8.2f}"
        for s in runs:
            per += f" {sum(x[1] for x in s.levels[i]) * 1e3 / max(len(s.levels[i]), 1):>8.2f}"
        print(per)
    for s in runs:
        kinds = {}
        for kind, a, b, nb in s.collectives:
            c = kinds.setdefault(kind, [0, 0])
            c[0] += 1
            c[1] += nb
        per = {k: (v[0] / len(roots), round(v[1] / len(roots) / 2**20, 3)) for k, v in kinds.items()}
        print(f"\nrank {s.rank}: levels exact vs the recorded {P}-rank run: {s.exact}; "
              f"collectives per traversal (calls, MiB received): {per}")
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"scale": args.scale, "P": P, "mode": args.mode, "roots": roots, "opts": opts,
                       "one_gpu": ref,
                       "ranks": [{"rank": s.rank, "exact": s.exact, "levels": s.levels, "wall_ms": s.wall_ms,
                                  "recorded_levels": s.recorded_levels, "collectives": s.collectives}
                                 for s in runs]}, f)
    return 0 if all(s.exact for s in runs) else 1


if __name__ == "__main__":
    sys.exit(main())
