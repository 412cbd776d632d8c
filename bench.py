#!/usr/bin/env python3
"""Headline benchmark: Graph500-style BFS GTEPS on RMAT-26 over N MI355X GPUs.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` -- for N > 1
launched with ``torch.distributed.run`` (one process per GPU; RANK, LOCAL_RANK,
WORLD_SIZE, MASTER_ADDR, MASTER_PORT from the environment).  One *step* = one
complete BFS traversal from a fresh random root (degree >= 1) on the fixed
RMAT-26 graph (strong scaling: the graph is 1D-partitioned over the N GPUs).
W untimed warm-up traversals, then EXACTLY K traversals timed between a
barrier + device synchronisation on both sides, max over ranks; rank 0 prints
one JSON line.  value = total traversed edges of the K traversals / timed wall
time (whole job, all GPUs).  The graph is generated on the GPUs with the
Graph500 Kronecker parameters (a=.57 b=.19 c=.19, edge factor 16, scrambled
vertex labels); weights/data are synthetic by construction (no dataset).

The reference (xxcclong/Distributed-CUDA-BFS) publishes no number
(BASELINE.md), so vs_baseline is null unless --baseline-gteps is given.
This process never imports torch: it uses the native core's own HIP runtime
and RCCL communicator.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "GTEPS (traversed edges/sec) on RMAT-26 + soc-LiveJournal1 at 1/2/4/8 MI355X"

# The reference publishes no number.  Its algorithm, re-implemented
# in HIP (`--mode ref`), measured on MI355X in this repo: (scale, n_gpus) -> GTEPS.
MEASURED_REF_GTEPS = {(26, 1): 0.8088}


def log(msg: str) -> None:
    print(f"[bench r{os.environ.get('RANK', '0')}] {msg}", file=sys.stderr, flush=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--graph", default=None, metavar="PATH",
                    help="real graph instead of RMAT: edge list / .mtx / binary .csr cache (e.g. soc-LiveJournal1; "
                         "no dataset ships with the repo and the GPU pool has no network)")
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--mode", default="do", choices=["ref", "td", "bu", "do", "simple", "scan"])
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--root-seed", type=int, default=12345)
    ap.add_argument("--alpha", type=float, default=24.0)
    ap.add_argument("--beta", type=float, default=96.0)
    ap.add_argument("--bu-lane-limit", type=int, default=8)
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="engine tuning option (see Engine.get_options()), repeatable")
    ap.add_argument("--no-hubs", action="store_true", help="bottom-up without the LDS hub frontier")
    ap.add_argument("--max-hubs", type=int, default=None)
    ap.add_argument("--device", default="hip", choices=["hip", "cpu"])
    ap.add_argument("--no-validate", action="store_true")
    ap.add_argument("--baseline-gteps", type=float, default=None)
    ap.add_argument("--per-level", action="store_true", help="print per-level records of the first timed run")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            log(f"--gpus {args.gpus} requested but WORLD_SIZE=1: launch with torch.distributed.run "
                f"--nproc-per-node {args.gpus}")
            return 2
    import distributed_cuda_bfs_amd as dbfs
    from distributed_cuda_bfs_amd.parallel.runtime import init_runtime
    from distributed_cuda_bfs_amd.utils.metrics import harmonic_mean

    N = dbfs.native
    rt = init_runtime(args.device)
    rank, nranks = rt.rank, rt.world
    log(f"backend {rt.backend.name}, comm {rt.comm.name}, ranks {nranks}")

    if args.graph:
        params = dbfs.read_graph(args.graph)  # every rank reads the file, shards its rows
        graph_name = os.path.basename(args.graph)
        n_vertices, n_input_edges = params.n, params.input_edges
    else:
        params = dbfs.rmat_params(args.scale, args.edge_factor, args.seed)
        graph_name = (f"RMAT-{args.scale} (Graph500 Kronecker a=.57 b=.19 c=.19, "
                      f"edge factor {args.edge_factor})")
        n_vertices, n_input_edges = params.n, params.m
    t0 = time.time()
    bfs = dbfs.BFS(params, rt, mode=args.mode, alpha=args.alpha, beta=args.beta,
                   bu_lane_limit=args.bu_lane_limit, hubs=not args.no_hubs, max_hubs=args.max_hubs)
    for kv in args.opt:
        name, _, val = kv.partition("=")
        bfs.engine.set_option(name, float(val))
    rt.backend.synchronize()
    rt.barrier()
    gen_s = time.time() - t0
    log(f"built {graph_name} shard: rows {bfs.graph.rows} nnz {bfs.graph.nnz} in {gen_s:.2f}s")

    roots = bfs.sample_roots(args.warmup + args.steps, seed=args.root_seed)
    if len(roots) < args.warmup + args.steps:
        log("could not sample enough roots")
        return 3
    warm, timed = roots[:args.warmup], roots[args.warmup:]

    validated = None
    for i, r in enumerate(warm):
        res = bfs.run(r)
        if i == 0 and not args.no_validate:
            validated = bfs.validate(r)
            log(f"validation of root {r}: {'OK' if validated else 'FAILED'}")
            if not validated:
                return 4
        log(f"warmup root {r}: {res.ms:.3f} ms, {res.gteps:.2f} GTEPS, depth {res.depth}")

    rt.barrier()
    rt.backend.synchronize()
    t_start = time.perf_counter()
    results = [bfs.run(r) for r in timed]
    rt.backend.synchronize()
    rt.barrier()
    wall_ms = (time.perf_counter() - t_start) * 1e3
    wall_ms = rt.comm.max_host(wall_ms)

    if rank == 0:
        for r in results:
            dirs = "".join(lv["dir"] for lv in r.levels)
            log(f"timed root {r.source}: {r.ms:.3f} ms {r.gteps:.1f} GTEPS levels {dirs} "
                f"frontier-edges {[lv['frontier_edges'] for lv in r.levels]}")
    edges = sum(r.edges for r in results)
    bfs_ms = sum(r.ms for r in results)
    value = edges / (wall_ms * 1e6)
    if args.per_level:
        # extra (untimed) traversals of the fastest and the slowest timed root with
        # per-level device events
        order = sorted(results, key=lambda r: r.ms)
        bfs.engine.phase_timing = True
        profs = [bfs.run(order[0].source), bfs.run(order[-1].source)]
        bfs.engine.phase_timing = False
        for prof in profs:
            if rank != 0:
                break
            log(f"per-level profile of root {prof.source} ({prof.ms:.3f} ms incl. event overhead):")
            for lv in prof.levels:
                log(f"  level {lv['level']} {lv['dir']} frontier {lv['frontier']} edges {lv['frontier_edges']}"
                    f" new {lv['discovered']} {lv['ms']:.3f} ms (collectives {lv.get('comm_ms', 0.0):.3f} ms)")
    # One extra (untimed) traversal of the median timed root with per-level
    # device events: where the time goes (collectives vs kernels) at this N.
    med = sorted(results, key=lambda r: r.ms)[len(results) // 2]
    bfs.engine.phase_timing = True
    prof = bfs.run(med.source)
    bfs.engine.phase_timing = False
    level_profile = [[lv["dir"], round(lv["ms"], 4), round(lv.get("comm_ms", 0.0), 4)] for lv in prof.levels]
    baseline = args.baseline_gteps
    if baseline is None and not args.graph and args.edge_factor == 16 and args.mode != "ref":
        baseline = MEASURED_REF_GTEPS.get((args.scale, nranks))
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "GTEPS",
            "n_gpus": nranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_ms / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": (round(value / baseline, 2) if baseline else None),
            "baseline": ("reference algorithm (--mode ref) on MI355X, BASELINE.md" if baseline else None),
            "dtype": "int32",
            "data": (f"file {graph_name}, random roots" if args.graph
                     else "synthetic (Graph500 RMAT generated on device, random roots)"),
            "config": {
                "model": graph_name,
                "global_batch": 1,
                "seq_len": None,
                "parallelism": f"1d-vertex-partition x{nranks}",
                "mode": args.mode,
                "vertices": n_vertices,
                "input_edges": n_input_edges,
                "directed_edges": bfs.engine.global_directed_edges,
            },
            "bfs_ms_mean": round(bfs_ms / len(results), 4),
            "harmonic_mean_gteps": round(harmonic_mean([r.gteps for r in results]), 4),
            "traversed_edges_mean": edges // len(results),
            "depth_mean": sum(r.depth for r in results) / len(results),
            "mispredicted_levels": sum(r.mispredicts for r in results),
            "validated": validated,
            "generate_s": round(gen_s, 3),
            "level_profile": {"root": med.source, "levels": level_profile,
                              "columns": ["dir", "ms", "comm_ms"]},
            # the timed traversal of the same root, from the device clock the
            # kernels stamp (device loop only): level time and the idle gap
            # before its first kernel
            "level_clock": {"levels": [[lv["dir"], round(lv["ms"], 4), round(lv.get("gap_ms", -1.0), 4)]
                                       for lv in med.levels],
                            "columns": ["dir", "ms", "gap_ms"]},
        }
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
