#!/usr/bin/env python3
"""Same-process A/B of one engine option's two values on the LiveJournal-sized
uniform and power-law graphs and RMAT-22 (top-down only by default): GTEPS
over K roots (alternating A/B passes, 3 each), every root validated, and for
one root the per-level device time (µs) of both.

  python tools/td_option_ab.py --option td_hub_edges --a 4096 --b 0 --roots 16
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--option", required=True)
    ap.add_argument("--a", type=float, default=1.0)
    ap.add_argument("--b", type=float, default=0.0)
    ap.add_argument("--roots", type=int, default=16)
    ap.add_argument("--root-seed", type=int, default=7)
    ap.add_argument("--mode", default="td")
    ap.add_argument("--graphs", default="lj,lj_pl,r22")
    ap.add_argument("--set", action="append", default=[], metavar="NAME=VALUE",
                    help="an engine option set on both sides")
    ap.add_argument("--device", default="hip")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()

    import distributed_cuda_bfs_amd as dbfs
    from distributed_cuda_bfs_amd.parallel.runtime import init_runtime

    rt = init_runtime(args.device)
    n, m, dmax = dbfs.ops.graph.LJ_SIZED_POWER_LAW
    graphs = {"lj": dbfs.uniform_params(n, m, 101), "lj_pl": dbfs.power_law_params(n, m, dmax, 201),
              "r22": dbfs.rmat_params(22, 16, 1), "r26": dbfs.rmat_params(26, 16, 1)}
    out = {}
    for name in args.graphs.split(","):
        bfs = dbfs.BFS(graphs[name], rt, mode=args.mode)
        for kv in args.set:
            k, v = kv.split("=", 1)
            bfs.engine.set_option(k, float(v))
        roots = bfs.sample_roots(args.roots, seed=args.root_seed)
        rec = {"a": [], "b": []}
        for _ in range(3):
            for side, v in (("a", args.a), ("b", args.b)):
                bfs.engine.set_option(args.option, v)
                bfs.run(roots[0])
                ms = edges = 0.0
                for r in roots:
                    res = bfs.run(r)
                    ms += res.ms
                    edges += res.edges
                rec[side].append(round(edges / (ms * 1e-3) / 1e9, 2))
        levels = {}
        for side, v in (("a", args.a), ("b", args.b)):
            bfs.engine.set_option(args.option, v)
            ok = True
            for r in roots:
                bfs.run(r)
                ok = ok and bfs.validate(r)
            bfs.engine.phase_timing = True
            res = bfs.run(roots[len(roots) // 2])
            bfs.engine.phase_timing = False
            levels[side] = [[lv["dir"], round(lv["ms"] * 1e3, 1), int(lv.get("frontier", -1))] for lv in res.levels]
            # chains: level, form, ranged (R) / unvisited filter (U) flags
            rec[side + "_chains"] = " ".join(f"{c[0]}{c[1]}{'R' if c[5] else ''}{'U' if c[6] else ''}{'/%d' % c[7] if c[7] > 1 else ''}"
                                             for c in res.chains)
            rec[side + "_valid"] = ok
        rec["levels_us"] = levels
        out[name] = rec
        print(f"{name} {args.mode} {args.option}={args.a}: {rec['a']} GTEPS  {args.option}={args.b}: {rec['b']} "
              f"valid {rec['a_valid']}/{rec['b_valid']}", flush=True)
        print(f"  levels a: {levels['a']}\n  levels b: {levels['b']}", flush=True)
        print(f"  chains a: {rec['a_chains']}\n  chains b: {rec['b_chains']}", flush=True)
        del bfs
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
    return 0 if all(r["a_valid"] and r["b_valid"] for r in out.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
