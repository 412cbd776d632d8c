"""Multi-process BFS on the CPU backend over torch.distributed (gloo).

One process per rank, exactly like the GPU deployment (one process per GPU),
with the communicator swapped for TorchComm -- the engine, partitioning and
collectives schedule are the production code.  Replaces the reference's
2-rank-only MPI path (bfs_mpi.cu:549-643), which was never actually validated
(its expected output was the GPU output).
"""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, scale, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
        import distributed_cuda_bfs_amd as dbfs
        from distributed_cuda_bfs_amd.parallel.runtime import init_runtime

        rt = init_runtime("cpu")
        assert rt.world == world and rt.rank == rank and rt.comm.name.startswith("torch")
        p = dbfs.rmat_params(scale, 16, 31)
        bfs = dbfs.BFS(p, rt, mode=mode)
        roots = bfs.sample_roots(3, seed=4)
        out = []
        for r in roots:
            res = bfs.run(r)
            out.append((r, bfs.levels(), res.reached, res.edges, bfs.validate(r)))
        q.put((rank, out))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback

        q.put((rank, "ERR " + repr(e) + traceback.format_exc()))


@pytest.mark.parametrize("world,mode", [(2, "do"), (2, "ref"), (3, "td"), (3, "bu"), (4, "simple")])
def test_gloo_multiprocess(world, mode):
    import multiprocessing as mp

    import distributed_cuda_bfs_amd as dbfs

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    scale = 10
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, scale, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        rank, out = q.get(timeout=240)
        assert not isinstance(out, str), out
        results[rank] = out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    csr = dbfs.host_csr_from_params(dbfs.rmat_params(scale, 16, 31))
    for rank, out in results.items():
        for src, lv, reached, edges, ok in out:
            exp, _ = dbfs.cpu_bfs(csr, src)
            assert np.array_equal(lv, exp), (rank, src)
            assert reached == int((exp != dbfs.UNREACHED).sum())
            assert ok
