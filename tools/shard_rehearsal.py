#!/usr/bin/env python3
"""Per-GPU shard sizing at a large graph's real shape, rehearsed on one GPU:
P virtual ranks (threads, one backend each, VirtualComm) each build their 1D
shard of a device-generated graph -- by default the Friendster-sized power-law
stand-in (65,608,366 V / 1,806,067,135 input edges, largest expected degree
5,214; BASELINE config 5) -- then traverse K random roots, every one checked by
the device Graph500 validator.  Reports every rank's rows, adjacency entries
and device bytes (DBufs of its backend, now and at peak), next to what the
reference's layout would need per GPU: the whole CSR and 8 int arrays of N
replicated on every device (bfs.cu:336-351), with int indices that cannot hold
this many entries (E >= 2^31).

  python tools/shard_rehearsal.py --ranks 8 --roots 4 --json out.json
  python tools/shard_rehearsal.py --ranks 8 --rmat 27            # config 4's graph

The traversals time-share one GPU, so their times are not P-GPU times (the
shadow ranks measure those); this checks that the sharded layout holds at the
real shape and what each GPU would hold.
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
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--roots", type=int, default=4)
    ap.add_argument("--root-seed", type=int, default=777)
    ap.add_argument("--rmat", type=int, default=None, help="RMAT scale instead of the Friendster-sized graph")
    ap.add_argument("--power-law", default=None, metavar="N:M:DMAX",
                    help="power-law graph shape (default: Friendster's, 65608366:1806067135:5214)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--mode", default="do")
    ap.add_argument("--device", default="hip")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()

    import distributed_cuda_bfs_amd as dbfs
    from distributed_cuda_bfs_amd.parallel.runtime import run_virtual_ranks

    if args.rmat:
        params = dbfs.rmat_params(args.rmat, 16, args.seed)
        graph = f"RMAT-{args.rmat} (Graph500, edge factor 16)"
    else:
        n, m, dmax = (int(x) for x in (args.power_law.split(":") if args.power_law
                                       else dbfs.ops.graph.FRIENDSTER_SIZED_POWER_LAW))
        params = dbfs.power_law_params(n, m, dmax, args.seed)
        graph = f"power-law (Chung-Lu, tail exponent 2.5, max expected degree {dmax}) {n} V / {m} E"
    P = args.ranks
    log = lambda s: print(f"[rehearsal] {s}", file=sys.stderr, flush=True)  # noqa: E731
    log(f"{graph}, {P} virtual ranks on one {args.device} device")

    def body(rt):
        t0 = time.time()
        b = dbfs.BFS(params, rt, mode=args.mode)
        rt.barrier()
        build_s = time.time() - t0
        built = rt.backend.device_bytes
        roots = b.sample_roots(args.roots, seed=args.root_seed)
        runs = []
        for r in roots:
            res = b.run(r)
            ok = b.validate(r)
            runs.append({"root": int(r), "ms": round(res.ms, 3), "reached": int(res.reached), "edges": int(res.edges),
                         "depth": int(res.depth), "levels": "".join(lv["dir"] for lv in res.levels),
                         "validated": bool(ok)})
            if rt.rank == 0:
                log(f"root {r}: reached {res.reached} edges {res.edges} depth {res.depth} "
                    f"{''.join(lv['dir'] for lv in res.levels)} validated {ok}")
        return {"rank": rt.rank, "rows": int(b.graph.rows), "nnz": int(b.graph.nnz), "build_s": round(build_s, 2),
                "device_bytes_after_build": int(built), "device_bytes": int(rt.backend.device_bytes),
                "peak_device_bytes": int(rt.backend.peak_device_bytes), "runs": runs,
                "total_directed": int(b.engine.global_directed_edges), "n": int(b.n)}

    t0 = time.time()
    outs = run_virtual_ranks(P, body, device=args.device)
    wall = time.time() - t0
    n = outs[0]["n"]
    E = outs[0]["total_directed"]
    ref_bytes = (E + 8 * n) * 4  # bfs.cu:336-344 per device: adjacency E ints + 8 arrays of N ints
    rec = {
        "graph": graph, "ranks": P, "device": args.device, "n": n, "directed_entries": E,
        "wall_s": round(wall, 1),
        "all_roots_validated": all(r["validated"] for o in outs for r in o["runs"]),
        "roots_agree": all(o["runs"] == outs[0]["runs"] or
                           [(r["reached"], r["edges"], r["depth"]) for r in o["runs"]] ==
                           [(r["reached"], r["edges"], r["depth"]) for r in outs[0]["runs"]] for o in outs),
        "per_rank": [{k: o[k] for k in ("rank", "rows", "nnz", "build_s", "device_bytes_after_build",
                                        "device_bytes", "peak_device_bytes")} for o in outs],
        "max_rank_peak_gb": round(max(o["peak_device_bytes"] for o in outs) / 2**30, 3),
        "reference_layout_per_gpu_gb": round(ref_bytes / 2**30, 3),
        "reference_layout_fits_int32": E < 2**31,
        "runs_rank0": outs[0]["runs"],
        "data": "synthetic (generated on the device); parity with the real dataset unpinned",
    }
    for o in rec["per_rank"]:
        log(f"rank {o['rank']}: rows {o['rows']} entries {o['nnz']} device {o['device_bytes'] / 2**30:.2f} GiB "
            f"(peak {o['peak_device_bytes'] / 2**30:.2f} GiB)")
    log(f"reference layout: {rec['reference_layout_per_gpu_gb']} GiB per GPU, int32 indices "
        f"{'fit' if rec['reference_layout_fits_int32'] else 'OVERFLOW'}; all roots validated "
        f"{rec['all_roots_validated']}")
    print(json.dumps(rec))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rec, f, indent=1)
    return 0 if rec["all_roots_validated"] else 1


if __name__ == "__main__":
    sys.exit(main())
