"""Failure detection: a failed, crashed or hung rank must turn
into an error on its peers, never a hang.  Faults are injected with
DBFS_FAULT_INJECT (Engine::inject_fault); collective waits are bounded by
DBFS_COMM_TIMEOUT_S.  All CPU: virtual ranks (threads) and multi-process CLI
runs over the TCP transport.  The RCCL watchdog (ncclCommGetAsyncError + wait
bound) is exercised by tests/test_gpu_engine.py on a GPU box."""
import os
import socket
import subprocess
import threading
import time

import pytest

import distributed_cuda_bfs_amd as dbfs
from distributed_cuda_bfs_amd.parallel.runtime import run_virtual_ranks

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BFS_BIN = os.path.join(REPO, "bin", "bfs")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(120)
@pytest.mark.parametrize("mode", ["do", "ref", "scan"])
def test_virtual_rank_failure_aborts_group(monkeypatch, mode):
    monkeypatch.setenv("DBFS_FAULT_INJECT", "rank=1,level=1,kind=throw")
    p = dbfs.rmat_params(10, 16, 3)

    def body(rt):
        bfs = dbfs.BFS(p, rt, mode=mode)
        bfs.run(bfs.sample_roots(1, seed=1)[0])
        return True

    with pytest.raises(Exception, match="injected fault"):
        run_virtual_ranks(3, body, device="cpu")


def test_fault_spec_validation(monkeypatch):
    monkeypatch.setenv("DBFS_FAULT_INJECT", "rank=0,level=1,kind=explode")
    with pytest.raises(Exception, match="kind must be"):
        dbfs.BFS(dbfs.rmat_params(8, 4, 1), dbfs.init_runtime("cpu"))
    monkeypatch.setenv("DBFS_FAULT_INJECT", "rank=0,depth=1")
    with pytest.raises(Exception, match="unknown key"):
        dbfs.BFS(dbfs.rmat_params(8, 4, 1), dbfs.init_runtime("cpu"))


def test_fault_on_other_rank_or_level_is_inert(monkeypatch):
    # the fault names a level the traversal never reaches: runs are unaffected
    monkeypatch.setenv("DBFS_FAULT_INJECT", "rank=0,level=999")
    p = dbfs.rmat_params(9, 8, 2)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, dbfs.init_runtime("cpu"))
    bfs.run(1)
    assert (bfs.levels() == dbfs.cpu_bfs(csr, 1)[0]).all()


@pytest.mark.timeout(60)
def test_virtual_barrier_times_out(monkeypatch):
    monkeypatch.setenv("DBFS_COMM_TIMEOUT_S", "0.5")
    rt = dbfs.init_runtime("cpu")
    group = dbfs.native.VirtualGroup(2)
    comm = dbfs.native.virtual_comm(group, 0, rt.backend)
    t0 = time.time()
    with pytest.raises(Exception, match="timed out"):
        comm.barrier()  # rank 1 never arrives
    assert time.time() - t0 < 10
    assert group.aborted


@pytest.mark.timeout(60)
def test_virtual_group_abort_wakes_waiters():
    rt = dbfs.init_runtime("cpu")
    group = dbfs.native.VirtualGroup(3)
    comms = [dbfs.native.virtual_comm(group, r, rt.backend) for r in range(2)]
    errs = []

    def wait(c):
        try:
            c.barrier()
        except Exception as e:  # noqa: BLE001
            errs.append(str(e))

    th = [threading.Thread(target=wait, args=(c,)) for c in comms]
    for t in th:
        t.start()
    time.sleep(0.2)
    group.abort("rank 2 crashed")
    for t in th:
        t.join(timeout=10)
    assert len(errs) == 2 and all("rank 2 crashed" in e for e in errs)


def _launch_cli(world, port, extra_env, args):
    procs = []
    for r in range(world):
        env = dict(os.environ, WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port - 1), DBFS_BOOTSTRAP_PORT=str(port), **extra_env)
        procs.append(subprocess.Popen([BFS_BIN] + args, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    return procs


def _finish(procs, timeout):
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()  # exact child PID
            o, e = p.communicate()
        outs.append((p.returncode, o, e))
    return outs


def test_multiprocess_tcp_cli_ok():
    port = _free_port()
    procs = _launch_cli(2, port, {}, ["--rmat", "10", "3", "--cpu", "--quiet", "--validate", "--mode", "do"])
    outs = _finish(procs, 120)
    for rc, o, e in outs:
        assert rc == 0, e


@pytest.mark.timeout(180)
def test_multiprocess_crashed_rank_is_detected():
    port = _free_port()
    procs = _launch_cli(2, port, {"DBFS_FAULT_INJECT": "rank=1,level=1,kind=exit"},
                        ["--rmat", "10", "3", "--cpu", "--quiet", "--mode", "do"])
    t0 = time.time()
    (rc0, _, e0), (rc1, _, e1) = _finish(procs, 120)
    assert rc1 == 17, e1
    assert rc0 != 0 and "closed the connection" in e0, e0
    assert time.time() - t0 < 100


@pytest.mark.timeout(180)
def test_multiprocess_hung_rank_times_out():
    port = _free_port()
    procs = _launch_cli(2, port, {"DBFS_FAULT_INJECT": "rank=1,level=1,kind=hang", "DBFS_COMM_TIMEOUT_S": "3"},
                        ["--rmat", "10", "3", "--cpu", "--quiet", "--mode", "do"])
    t0 = time.time()
    rc0_out = _finish(procs[:1], 90)[0]
    elapsed = time.time() - t0
    procs[1].kill()  # the hung rank (exact PID)
    procs[1].communicate()
    rc0, _, e0 = rc0_out
    assert rc0 != 0 and "timed out" in e0, e0
    assert elapsed < 60


@pytest.mark.timeout(60)
def test_bootstrap_and_collective_timeouts_are_separate(monkeypatch):
    """The TCP bootstrap's own exchanges wait DBFS_BOOTSTRAP_TIMEOUT_S (setup:
    a peer may still be ingesting its shard), TcpComm's collectives
    DBFS_COMM_TIMEOUT_S; each timeout names its setting.  Rank 1 connects and
    then never joins an exchange."""
    from distributed_cuda_bfs_amd._native import N

    monkeypatch.setenv("DBFS_BOOTSTRAP_TIMEOUT_S", "1.0")
    monkeypatch.setenv("DBFS_COMM_TIMEOUT_S", "0.3")
    port = _free_port()
    boots = [None, None]

    def make(r):
        boots[r] = N.TcpBootstrap("127.0.0.1", port, r, 2, 20.0)

    th = [threading.Thread(target=make, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
    b0 = boots[0]
    t0 = time.time()
    with pytest.raises(Exception, match="DBFS_BOOTSTRAP_TIMEOUT_S"):
        b0.allgather(b"x")
    assert 0.8 < time.time() - t0 < 10
    comm = N.tcp_comm(b0, dbfs.init_runtime("cpu").backend)
    t0 = time.time()
    with pytest.raises(Exception, match="DBFS_COMM_TIMEOUT_S"):
        comm.barrier()
    assert time.time() - t0 < 0.9
