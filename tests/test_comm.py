"""Communicator unit tests: alltoall, alltoallv with empty /
skewed / all-to-one patterns, allgather, allreduce -- for every host-testable
Comm implementation: VirtualComm (threads), TcpComm (processes, TCP bootstrap)
and TorchComm (processes, torch.distributed gloo).  The RCCL communicator runs
the same exercise in tests/test_gpu_engine.py (1 rank) and on the 8-GPU node.
"""
import os
import socket

import numpy as np
import pytest

import distributed_cuda_bfs_amd as dbfs
from distributed_cuda_bfs_amd.parallel.runtime import run_virtual_ranks

N = dbfs.native


def _patterns(P):
    """(name, counts[src][dst]) traffic matrices."""
    rng = np.random.default_rng(P)
    return [
        ("uniform", [[3] * P for _ in range(P)]),
        ("empty", [[0] * P for _ in range(P)]),
        ("skewed", [[int(x) for x in rng.integers(0, 9, P)] for _ in range(P)]),
        ("all_to_one", [[(7 if d == 0 else 0) for d in range(P)] for _ in range(P)]),
        ("self_only", [[(5 if d == s else 0) for d in range(P)] for s in range(P)]),
    ]


def _expected_alltoallv(P, counts, me):
    out = []
    for s in range(P):
        out += [s * 1000 + me * 100 + k for k in range(counts[s][me])]
    return out


def _exercise(comm, be, P, me):
    res = {}
    res["allreduce"] = N.comm_exercise(comm, be, "allreduce", np.array([me + 1, 10 * me, -me], np.int64)).tolist()
    res["allgather"] = N.comm_exercise(comm, be, "allgather", np.array([me, me * me], np.int64)).tolist()
    a2a_in = np.array([me * 100 + d for d in range(P) for _ in range(2)], np.int64)
    res["alltoall"] = N.comm_exercise(comm, be, "alltoall", a2a_in).tolist()
    for name, counts in _patterns(P):
        send = [s for d in range(P) for s in [me * 1000 + d * 100 + k for k in range(counts[me][d])]]
        out = N.comm_exercise(comm, be, "alltoallv", np.array(send, np.int64), [counts[me][d] for d in range(P)],
                              [counts[s][me] for s in range(P)])
        res["v_" + name] = out.tolist()
    return res


def _check(res, P, me):
    assert res["allreduce"] == [P * (P + 1) // 2, 10 * P * (P - 1) // 2, -P * (P - 1) // 2]
    assert res["allgather"] == [x for r in range(P) for x in (r, r * r)]
    assert res["alltoall"] == [s * 100 + me for s in range(P) for _ in range(2)]
    for name, counts in _patterns(P):
        assert res["v_" + name] == _expected_alltoallv(P, counts, me), name


@pytest.mark.parametrize("P", [1, 2, 3, 5])
def test_virtual_comm(P):
    def body(rt):
        return _exercise(rt.comm, rt.backend, P, rt.rank)

    for me, res in enumerate(run_virtual_ranks(P, body, device="cpu")):
        _check(res, P, me)


def test_local_comm():
    be = N.cpu_backend()
    _check(_exercise(N.local_comm(be), be, 1, 0), 1, 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _proc(kind, rank, world, port, q):
    try:
        import distributed_cuda_bfs_amd as d

        be = d.native.cpu_backend()
        if kind == "tcp":
            boot = d.native.TcpBootstrap("127.0.0.1", port, rank, world, 60.0)
            comm = d.native.tcp_comm(boot, be)
        else:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            import torch.distributed as dist

            dist.init_process_group("gloo", rank=rank, world_size=world)
            from distributed_cuda_bfs_amd.parallel.torch_comm import TorchComm

            comm = TorchComm()
        comm.bind_backend(be)
        assert comm.rank == rank and comm.size == world
        q.put((rank, _exercise(comm, be, world, rank)))
        comm.barrier()
    except Exception as e:  # pragma: no cover - reported by the parent
        import traceback

        q.put((rank, "ERR " + repr(e) + traceback.format_exc()))


@pytest.mark.parametrize("kind,world", [("tcp", 2), ("tcp", 4), ("torch", 3)])
def test_process_comms(kind, world):
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_proc, args=(kind, r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for rank, res in out.items():
        assert not isinstance(res, str), res
        _check(res, world, rank)


def test_bootstrap_ignores_a_silent_stray_connection():
    """A connection that never sends the hello (a port scanner, a stale
    client) is dropped after the short hello timeout instead of stalling rank
    0's accept loop for the whole collective timeout."""
    import socket
    import threading
    import time

    N = dbfs.native
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    boots = [None, None]

    def r0():
        boots[0] = N.TcpBootstrap("127.0.0.1", port, 0, 2, 60.0)

    t = threading.Thread(target=r0)
    t.start()
    stray = None
    for _ in range(200):  # rank 0 listening
        try:
            stray = socket.create_connection(("127.0.0.1", port), timeout=1)
            break
        except OSError:
            time.sleep(0.05)
    assert stray is not None
    t0 = time.time()
    boots[1] = N.TcpBootstrap("127.0.0.1", port, 1, 2, 60.0)
    t.join(timeout=60)
    assert not t.is_alive() and boots[0] is not None
    assert time.time() - t0 < 30
    stray.close()


def test_rccl_fallback_keeps_the_bootstrap_aligned():
    """A failed RCCL setup (here: no GPU, so rank 0 cannot make the id; on a
    shared GPU: the device check) is agreed over the bootstrap and every rank
    falls back to the inner communicator with the bootstrap's collective
    sequence intact -- the id broadcast happens on every rank before anything
    can fail (a desync here once surfaced as a TcpComm count mismatch)."""
    import socket
    import threading

    from distributed_cuda_bfs_amd.parallel.runtime import _rccl_or

    N = dbfs.native
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = [None, None]

    class FakeBackend:
        device_id = 0

    class Inner:
        name = "tcp"

    def body(r):
        boot = N.TcpBootstrap("127.0.0.1", port, r, 2, 60.0)
        inner = Inner()
        got = _rccl_or(inner, boot, FakeBackend(), r, 2, r)
        out[r] = (got is inner, [bytes(x) for x in boot.allgather(b"after%d" % r)])

    ts = [threading.Thread(target=body, args=(r,)) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    assert all(o == (True, [b"after0", b"after1"]) for o in out), out


def test_group_bootstrap_threads():
    """The in-process bootstrap (GroupBootstrap: the ranks of a VirtualGroup,
    one thread each) gathers every rank's bytes in rank order, broadcasts the
    root's and shares the group with its virtual communicators."""
    import threading

    from distributed_cuda_bfs_amd._native import N

    P = 4
    group = N.VirtualGroup(P)
    got = [None] * P

    def body(r):
        b = N.group_bootstrap(group, r)
        assert b.in_process and b.rank == r and b.size == P
        a = b.allgather(bytes([r]) * (r + 1))
        c = b.broadcast(b"root%d" % r, root=2)
        b.barrier()
        d = b.allgather(b"")
        got[r] = (a, c, d)

    th = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
    for r in range(P):
        a, c, d = got[r]
        assert a == [bytes([q]) * (q + 1) for q in range(P)]
        assert c == b"root2" and d == [b""] * P
