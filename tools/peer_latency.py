#!/usr/bin/env python3
"""Collective latency of the rank communicator (peer transport by default):
back-to-back collectives of several sizes, mean microseconds each.  Spawns
--ranks processes itself (all on DBFS_DEVICE, or one GPU per rank):
    python3 tools/peer_latency.py --ranks 2 [--ops allreduce allgather]"""
import argparse
import json
import os
import socket
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--ops", nargs="+", default=["allreduce", "allgather", "alltoall"])
    ap.add_argument("--sizes", type=int, nargs="+", default=[16, 8208, 65552, 1 << 20])
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        procs = []
        for r in range(args.ranks):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.ranks),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
        rc = 0
        for p in procs:
            rc = p.wait() or rc
        return rc
    import distributed_cuda_bfs_amd as dbfs
    from distributed_cuda_bfs_amd.parallel.runtime import init_runtime
    rt = init_runtime("hip")
    out = {}
    for op in args.ops:
        for b in args.sizes:
            out[f"{op}/{b}"] = round(dbfs.native.comm_latency(rt.comm, rt.backend, op, b, args.iters), 2)
    if rt.rank == 0:
        print(json.dumps({"comm": rt.comm.name, "ranks": rt.world, "us": out}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
