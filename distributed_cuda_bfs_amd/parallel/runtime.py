"""Per-process runtime: one backend (GPU or CPU) plus the rank's communicator.

Execution models:
  * one process per GPU (``torch.distributed.run`` / any launcher exporting
    RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT) -> the peer-memory
    communicator (IPC windows over xGMI) with a TCP inner communicator for its
    setup agreements; RCCL (bounded setup) only when the windows are
    unavailable, or with DBFS_COMM=rccl (the reference used CUDA-aware MPI,
    bfs_mpi.cu:800-808);
  * one process, P virtual ranks as threads on one device -> ``run_virtual_ranks``;
  * CPU multi-process over torch.distributed/gloo -> ``TorchComm``.
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass
from typing import Any, Callable, List, Optional

from .._native import N


@dataclass
class Runtime:
    backend: Any
    comm: Any
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    # the communicator a peer-memory communicator wraps (TCP), kept as the
    # fallback transport (bench.py --allow-fallback re-measures on it if a
    # traversal over the windows fails validation)
    fallback_comm: Any = None

    @property
    def is_gpu(self) -> bool:
        return bool(self.backend.is_gpu)

    def barrier(self) -> None:
        self.comm.barrier()


def _env_int(k: str, d: int) -> int:
    v = os.environ.get(k)
    return int(v) if v not in (None, "") else d


def _torch_dist_ready() -> bool:
    """True only if torch is already imported AND a process group exists (this
    module never imports torch itself: GPU processes keep a single HIP runtime)."""
    import sys

    dist = sys.modules.get("torch.distributed")
    return bool(dist is not None and dist.is_available() and dist.is_initialized())


def make_backend(device: str = "auto", local_rank: int = 0):
    if device == "auto":
        device = "hip" if N.hip_device_count() > 0 else "cpu"
    if device in ("hip", "gpu", "cuda"):
        return N.hip_backend(local_rank)
    if device == "cpu":
        return N.cpu_backend()
    raise ValueError(f"unknown device {device!r} (hip|cpu|auto)")


def init_runtime(device: str = "auto", comm: Optional[Any] = None) -> Runtime:
    """Create this process's backend and communicator from the launcher's environment."""
    world = _env_int("WORLD_SIZE", 1)
    rank = _env_int("RANK", 0)
    local_rank = _env_int("LOCAL_RANK", rank if world > 1 else 0)
    # DBFS_DEVICE pins every rank to one device id (debug: several ranks on one GPU).
    backend = make_backend(device, _env_int("DBFS_DEVICE", local_rank))
    fallback = None
    if comm is None:
        kind = os.environ.get("DBFS_COMM", "")
        if world == 1:
            comm = N.local_comm(backend)
        elif kind == "torch" or (not kind and not backend.is_gpu and _torch_dist_ready()):
            from .torch_comm import TorchComm
            comm = TorchComm()
        else:
            addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
            port = _env_int("DBFS_BOOTSTRAP_PORT", _env_int("MASTER_PORT", 29500) + 1)
            boot = N.TcpBootstrap(addr, port, rank, world)
            shared = "DBFS_DEVICE" in os.environ  # several ranks on one GPU (tests)
            if kind == "tcp" or (not kind and not backend.is_gpu):
                comm = N.tcp_comm(boot, backend)  # host collectives (CPU runs / debug fallback)
            elif kind == "rccl":
                comm = _make_rccl(boot, backend, rank, world, local_rank)
            else:
                # the peer-memory transport over a TCP inner communicator: the
                # windows carry every payload (slot-sized rounds), so TCP only
                # agrees setup steps -- no library collective stands between a
                # run and its first multi-GPU level
                inner = N.tcp_comm(boot, backend)
                comm, fallback = _try_peer(boot, backend, inner, rank, kind == "peer")
                if comm is inner and (not shared or os.environ.get("DBFS_TRY_RCCL") == "1"):
                    # no peer windows: RCCL over xGMI (bounded setup), else TCP
                    # (DBFS_TRY_RCCL=1: also on a shared GPU, where RCCL must
                    # fail -- tests of the agreed fallback)
                    comm = _rccl_or(inner, boot, backend, rank, world, local_rank)
    comm.bind_backend(backend)
    rt = Runtime(backend=backend, comm=comm, rank=comm.rank, world=comm.size, local_rank=local_rank)
    rt.fallback_comm = fallback
    return rt


def _make_rccl(boot, backend, rank: int, world: int, local_rank: int):
    """An RCCL communicator (one GPU per rank: the backend made LOCAL_RANK
    current before the communicator is created); its setup is bounded
    (DBFS_RCCL_INIT_TIMEOUT_S, native NcclComm)."""
    # every rank takes part in the id broadcast before anything can fail (an
    # empty id tells the others rank 0 could not make one), so the bootstrap's
    # collective sequence stays aligned for the agreement after a failure
    uid, why = b"", ""
    if rank == 0:
        try:
            uid = N.nccl_unique_id()
        except Exception as e:  # noqa: BLE001 - re-raised after the broadcast
            why = str(e) or type(e).__name__
    uid = boot.broadcast(uid)
    if not uid:
        raise RuntimeError(why or "rank 0 could not create the RCCL id")
    if backend.device_id != local_rank:
        raise RuntimeError(f"rank {rank}: backend on device {backend.device_id}, expected LOCAL_RANK {local_rank}")
    return N.nccl_comm(uid, rank, world, backend)  # RCCL over xGMI


def _rccl_or(inner, boot, backend, rank: int, world: int, local_rank: int):
    """RCCL if every rank builds it (agreed over the bootstrap), else `inner`."""
    import sys

    rc, err = None, ""
    try:
        rc = _make_rccl(boot, backend, rank, world, local_rank)
    except Exception as e:  # noqa: BLE001 - agreed below
        err = str(e) or type(e).__name__
    errs = [e for e in boot.allgather(err.encode()) if e]
    if not errs:
        return rc
    rc = None  # (a rank that built it drops it: every rank takes the same transport)
    if rank == 0:
        print(f"[dbfs] RCCL unavailable ({errs[0].decode(errors='replace')}); using {inner.name}",
              file=sys.stderr, flush=True)
    return inner


def _try_peer(boot, backend, inner, rank: int, required: bool):
    """The peer-memory communicator over `inner` if every rank can map every
    window and its self-test passes on every rank (the verdict is agreed), else
    `inner`.  Returns (comm, fallback)."""
    import sys

    slot = _env_int("DBFS_PEER_SLOT_MB", 16) << 20
    if os.environ.get("DBFS_PEER_SLOT_KB"):
        # small slots: large collectives go through the windows in slot-sized rounds (tests)
        slot = _env_int("DBFS_PEER_SLOT_KB", 0) << 10
    try:
        pc = N.peer_comm(boot, backend, inner, slot)
        ok, why = pc.self_test()
    except Exception as e:  # noqa: BLE001 - agreed on every rank by the native code
        ok, why, pc = False, str(e), None
    if ok:
        return pc, inner
    if required:
        raise RuntimeError(f"DBFS_COMM=peer: peer communicator unavailable: {why}")
    if rank == 0:
        print(f"[dbfs] peer communicator unavailable ({why}); using {inner.name}", file=sys.stderr, flush=True)
    return inner, None


def run_virtual_ranks(nranks: int, fn: Callable[[Runtime], Any], device: str = "auto",
                      device_id: int = 0) -> List[Any]:
    """Run ``fn(runtime)`` for P virtual ranks (threads) sharing one device.

    All ranks run the real partitioned code path (shards, owner routing,
    collectives); only the transport is an in-process copy.
    """
    group = N.VirtualGroup(int(nranks))
    rts = []
    for r in range(nranks):
        be = make_backend(device, device_id)
        rts.append(Runtime(backend=be, comm=N.virtual_comm(group, r, be), rank=r, world=nranks))
    out: List[Any] = [None] * nranks
    errs: List[Optional[BaseException]] = [None] * nranks

    def body(r: int) -> None:
        try:
            out[r] = fn(rts[r])
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errs[r] = e
            # wake the peers blocked in a collective (they raise too)
            group.abort(f"rank {r}: {e}")

    th = [threading.Thread(target=body, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    # report the root cause: the first rank whose failure was not a peer abort
    first = [e for e in errs if e is not None]
    if first:
        roots = [e for e in first if "virtual rank group aborted" not in str(e)]
        raise (roots or first)[0]
    return out
