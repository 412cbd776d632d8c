#!/usr/bin/env python3
"""Per-level device-clock times of REAL ranks (one process each, the peer
transport) for chosen roots -- to set against the shadow replay of the same
roots (tools/shadow_rank.py), which runs one rank's recorded kernels alone.

  python3 tools/real_ranks_levels.py --ranks 2 --scale 26 --root-list 8766153 13702079 --out gpurun_out/rr

Self-spawns --ranks processes (RANK / WORLD_SIZE env, 127.0.0.1 rendezvous);
with DBFS_DEVICE=0 they share one GPU (the peer windows then run the split
waits: a one-wave pre-wait launch per direct exchange, unfused collectives --
so each real level carries those launches and the other rank's kernels compete
for the CUs; the replay has neither).  Rank r writes <out>_r<r>.json: per root
the levels [dir, device ms, frontier edges] of the second of two runs.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn(n: int, argv, timeout_s: float) -> int:
    port, boot = _free_port(), _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DBFS_BOOTSTRAP_PORT=str(boot), DBFS_SPAWNED="1")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    t0 = time.time()
    while any(p.poll() is None for p in procs):
        if time.time() - t0 > timeout_s or any(p.poll() not in (None, 0) for p in procs):
            time.sleep(20)
            for p in procs:
                if p.poll() is None:
                    p.kill()
            break
        time.sleep(0.1)
    codes = [p.wait() for p in procs]
    return next((c for c in codes if c), 0)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--root-list", type=int, nargs="+", required=True)
    ap.add_argument("--out", default="gpurun_out/rr")
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--timeout", type=float, default=500.0)
    ap.add_argument("--device", default="hip")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ:
        return spawn(args.ranks, sys.argv[1:], args.timeout)

    import distributed_cuda_bfs_amd as dbfs
    from distributed_cuda_bfs_amd.parallel.runtime import init_runtime

    rt = init_runtime(args.device)
    bfs = dbfs.BFS(dbfs.rmat_params(args.scale, 16, 1), rt, mode="do")
    for kv in args.opt:
        k, _, v = kv.partition("=")
        bfs.engine.set_option(k, float(v))
    out = {"rank": rt.rank, "world": rt.world, "comm": rt.comm.name, "roots": {}}
    for r in args.root_list:
        bfs.run(r)
        res = bfs.run(r)
        out["roots"][str(r)] = {"ms": res.ms, "levels": [[lv["dir"], lv["ms"], lv["frontier_edges"]] for lv in res.levels],
                                "chains": [c[:2] for c in res.chains]}
    with open(f"{args.out}_r{rt.rank}.json", "w") as f:
        json.dump(out, f)
    rt.barrier()
    return 0


if __name__ == "__main__":
    sys.exit(main())
