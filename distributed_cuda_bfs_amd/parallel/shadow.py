"""Shadow rank: the per-rank cost of a P-GPU traversal, measured on one GPU.

A P-rank job cannot run on a one-GPU box, and P virtual ranks sharing the GPU
only show their kernels interleaved.  Instead:

1. **record** -- P virtual ranks (threads on one device) run the traversals;
   the communicator of every rank of interest is wrapped in a ``RecordComm``
   that keeps each collective's output (remote frontier slices, candidate
   slices / lists, all-reduced totals) on the host, in call order;
2. **replay** -- rank r is then built alone (its shard of the same graph) on
   the same device with a ``ReplayComm`` of its tape: each collective writes
   the recorded output with one device copy, so rank r's kernels see exactly
   the inputs of the P-rank run, with the whole GPU to themselves.

The replayed traversal's per-level device-clock times are the compute (plus
launch gaps and one device copy per collective) of rank r in a P-GPU run --
what replaces the launch-per-device + synchronize step of the reference
(bfs.cu:577-591, bfs_mpi.cu:586-593) -- and its levels are checked against the
recorded run's.  Communication is then added from the tapes' byte counts and a
link model (utils/comm_model.py).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from .._native import N
from .runtime import Runtime, make_backend


@dataclass
class ShadowRun:
    """One rank's replayed traversals (and the recorded run they reproduce)."""
    rank: int
    nranks: int
    roots: List[int]
    # per root: [(dir, device-clock ms, frontier edges)] of the replayed traversal
    levels: List[List[tuple]] = field(default_factory=list)
    wall_ms: List[float] = field(default_factory=list)
    recorded_levels: List[List[tuple]] = field(default_factory=list)
    exact: bool = True
    tape_records: int = 0
    tape_bytes: int = 0
    collectives: List[tuple] = field(default_factory=list)  # (kind, a, b, bytes) of the traversals


def _engine_opts(bfs, opts: Optional[Dict[str, float]]) -> None:
    for k, v in (opts or {}).items():
        bfs.engine.set_option(k, float(v))


def shadow_ranks(graph: Any, nranks: int, ranks: Sequence[int], roots: Sequence[int], mode: str = "do",
                 device: str = "auto", device_id: int = 0, warmup: int = 1,
                 opts: Optional[Dict[str, float]] = None, bfs_kwargs: Optional[Dict[str, Any]] = None
                 ) -> List[ShadowRun]:
    """Record a ``nranks``-rank run of ``roots`` (after ``warmup`` untimed
    traversals of the first root) and replay every rank in ``ranks`` alone.
    ``graph``: GenParams or HostCSR (every rank builds its own shard)."""
    from ..models.bfs import BFS

    ranks = sorted(set(int(r) for r in ranks))
    for r in ranks:
        if not 0 <= r < nranks:
            raise ValueError(f"rank {r} outside [0, {nranks})")
    bfs_kwargs = dict(bfs_kwargs or {})
    roots = [int(r) for r in roots]
    plan = [roots[0]] * warmup + roots

    # ---- 1. record (P virtual ranks) --------------------------------------------
    group = N.VirtualGroup(int(nranks))
    rts, recs = [], {}
    for r in range(nranks):
        be = make_backend(device, device_id)
        comm = N.virtual_comm(group, r, be)
        if r in ranks:
            comm = N.record_comm(comm, be)
            recs[r] = comm
        rts.append(Runtime(backend=be, comm=comm, rank=r, world=nranks))
    recorded: Dict[int, List[List[tuple]]] = {}
    levels_rec: Dict[int, np.ndarray] = {}
    errs: List[Optional[BaseException]] = [None] * nranks

    def body(r: int) -> None:
        try:
            bfs = BFS(graph, rts[r], mode=mode, **bfs_kwargs)
            _engine_opts(bfs, opts)
            out = []
            for src in plan:
                res = bfs.run(src)
                out.append([(lv["dir"], lv["ms"], lv["frontier_edges"]) for lv in res.levels])
            if r in ranks:
                recorded[r] = out[warmup:]
                levels_rec[r] = np.asarray(bfs.local_levels()).copy()  # the last root's owned levels
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errs[r] = e
            group.abort(f"rank {r}: {e}")

    th = [threading.Thread(target=body, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    first = [e for e in errs if e is not None]
    if first:
        roots_err = [e for e in first if "virtual rank group aborted" not in str(e)]
        raise (roots_err or first)[0]
    tapes = {r: recs[r].tape for r in ranks}
    del rts, recs

    # ---- 2. replay each rank alone --------------------------------------------------
    out: List[ShadowRun] = []
    for r in ranks:
        be = make_backend(device, device_id)
        comm = N.replay_comm(tapes[r], be)
        rt = Runtime(backend=be, comm=comm, rank=r, world=nranks)
        bfs = BFS(graph, rt, mode=mode, **bfs_kwargs)
        _engine_opts(bfs, opts)
        sr = ShadowRun(rank=r, nranks=nranks, roots=roots, tape_records=len(tapes[r]), tape_bytes=tapes[r].bytes)
        pos0 = None
        for i, src in enumerate(plan):
            if i == warmup:
                pos0 = comm.position
            res = bfs.run(src)
            if i >= warmup:
                sr.levels.append([(lv["dir"], lv["ms"], lv["frontier_edges"]) for lv in res.levels])
                sr.wall_ms.append(res.ms)
        be.synchronize()
        if comm.position != len(comm):
            raise RuntimeError(f"rank {r}: the replay consumed {comm.position} of {len(comm)} recorded collectives")
        sr.collectives = [tuple(x) for x in tapes[r].records()[pos0:]] if pos0 is not None else []
        sr.recorded_levels = recorded[r]
        got = np.asarray(bfs.local_levels())
        sr.exact = bool(np.array_equal(got, levels_rec[r])) and all(
            [d for d, _, _ in a] == [d for d, _, _ in b] and [m for _, _, m in a] == [m for _, _, m in b]
            for a, b in zip(sr.levels, sr.recorded_levels))
        out.append(sr)
        del bfs, comm, rt
    return out
