"""Per-level communication model of the multi-rank device loop.

Mirrors what ``Engine::run_bitmap_device`` (csrc/engine/engine.cpp,
``enqueue_level`` / ``finish_ranks``) issues for each level chain, so the
collectives and bytes of a traversal can be predicted from its chains
(``BFSResult.chains``: level, form, capacity, gather, pushed frontier,
unvisited filter, split parts, hub cut)
and checked against the
communicators' traffic counters (``Comm.traffic()``, tests/test_comm_model.py).
``table`` turns a 1-GPU level profile into the per-level bytes / collectives
table of docs/ARCHITECTURE.md §4.

One collective per level, plus the payload a top-down level must move:

* every chain ends with ONE collective: the level's totals all-reduced and --
  when the next level is predicted bottom-up -- its output frontier slice
  all-gathered in the same launch (``Comm.allgather_allreduce``);
* a sparse top-down chain (``S``) exchanges owner lists, count-sized on the
  peer transport (accounted here, as by the counters, at the lists' capacity);
* a dense top-down chain (``T``) exchanges candidate bitmap slices;
* a bottom-up chain (``B``) whose input frontier was not gathered by the
  previous collective (a mispredicted switch) gathers it itself; one with the
  hub cut's launches exchanges its remote claims as bitmap slices.

Bytes are what one rank sends to the other ranks under a direct exchange:
alltoall / allgather (P - 1) x the per-peer bytes, all-reduce (P - 1) x the
vector, alltoallv the counts to other ranks.

Reference being replaced: the per-level exchange of bfs.cu:587-609 (owner
buckets copied peer to peer after a count exchange, then a host sum) and
bfs_mpi.cu:601-621 (Sendrecv + Allreduce).
"""
from __future__ import annotations

from collections import Counter
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence, Tuple

WORD = 8  # bytes per bitmap word (64 vertices)


@dataclass
class ModelConfig:
    nranks: int
    slice_words: int              # Partition.slice_words(): words of one rank's bitmap slice
    mode: str = "do"              # engine mode: do / td / bu
    fused: bool = False           # the transport runs allgather_allreduce as one launch (peer windows, RCCL group)
    list_form_edges: int = 1 << 21  # EngineOptions.list_form_edges

    @property
    def list_max(self) -> int:
        """The owner lists' capacity: list_form_edges, at most a rank's part
        (a sparse chain recorded with cap 0 exchanges lists of this size)."""
        return min(self.list_form_edges, self.slice_words * 64)


@dataclass
class ChainTraffic:
    calls: Counter = field(default_factory=Counter)
    bytes: Counter = field(default_factory=Counter)

    def add(self, kind: str, nbytes: int) -> None:
        self.calls[kind] += 1
        self.bytes[kind] += int(nbytes)

    def merge(self, o: "ChainTraffic") -> None:
        self.calls.update(o.calls)
        self.bytes.update(o.bytes)

    @property
    def total_bytes(self) -> int:
        return sum(self.bytes.values())

    @property
    def total_calls(self) -> int:
        """Collective launches (fused ones count once)."""
        return sum(v for k, v in self.calls.items() if k not in ("barrier", "fused")) - self.calls["fused"]


def level_end(cfg: ModelConfig, gather: bool, push: bool = False) -> ChainTraffic:
    """The one collective that ends a level (or the seed).  A pushed frontier (push: the producing kernels store the slices into the
    peers' windows, Comm::direct_frontier) is accounted as an all-gather of its
    own -- the same bytes, no launch fused with the totals."""
    P, W = cfg.nranks, cfg.slice_words
    t = ChainTraffic()
    if gather:
        t.add("allgather", (P - 1) * W * WORD)
    t.add("allreduce", (P - 1) * 8 * 2)
    if gather and cfg.fused and not push:
        t.add("fused", 0)
    return t


def chain_traffic(cfg: ModelConfig, form: str, cap: int, gather: bool, in_gathered: bool,
                  push: bool = False, cut: bool = False) -> ChainTraffic:
    """Collectives of one level chain."""
    P, W = cfg.nranks, cfg.slice_words
    t = ChainTraffic()
    if form == "B" and not in_gathered:
        t.add("allgather", (P - 1) * W * WORD)              # input frontier slices (+ visited merge)
    if form == "B" and cut and P > 1:
        t.add("alltoall", (P - 1) * W * WORD)               # the hub cut's remote claims
    if form == "S":
        t.add("alltoallv", (P - 1) * ((cap or cfg.list_max) + 1) * 4)  # owner lists, count first
    elif form == "T":
        t.add("alltoall", (P - 1) * W * WORD)               # candidate bitmap slices
    t.merge(level_end(cfg, gather, push))
    return t


def run_traffic(cfg: ModelConfig, chains: Iterable[Tuple]) -> ChainTraffic:
    """Traffic of one traversal from its enqueued chains (level, form, cap,
    gather[, push, unvis, split, cut]): start barrier, every chain, the wall-time max at
    the end.  (The seed needs no collective: every rank seeds the traversal
    from its replicated degree array, and writes a bottom-up first level's
    whole seed frontier itself.)"""
    P = cfg.nranks
    tot = ChainTraffic()
    tot.add("barrier", 0)
    seed_gather = cfg.mode == "bu"
    gathered = {-1: seed_gather}
    for level, form, cap, gather, *more in chains:
        tot.merge(chain_traffic(cfg, form, int(cap), bool(gather), gathered.get(level - 1, False),
                                bool(more[0]) if more else False, bool(more[3]) if len(more) > 3 else False))
        gathered[level] = bool(gather)
    tot.add("allgather", (P - 1) * 8)  # max over ranks of the wall time
    return tot


def predicted_forms(levels: Sequence[Tuple[str, int]], cfg: ModelConfig, list_form_edges: int = 1 << 21,
                    xsparse_edges: int = 1 << 20) -> List[Tuple[int, str, int, bool]]:
    """Chains of a perfectly predicted traversal with per-level (direction,
    frontier edges), plus the trailing no-op chain the loop enqueues ahead."""
    seq = list(levels) + [("T", 0)]
    lim = min(xsparse_edges, list_form_edges) if cfg.mode != "bu" else -1
    out = []
    for L, (d, mf) in enumerate(seq):
        nxt = seq[L + 1][0] if L + 1 < len(seq) else "T"
        gather = nxt == "B"
        if d == "B":
            out.append((L, "B", 0, gather))
        elif list_form_edges > 0 and mf <= lim:
            out.append((L, "S", list_form_edges, gather))
        else:
            out.append((L, "T", 0, gather))
    return out


def table(levels: Sequence[Tuple[str, int]], n: int, nranks: int, mode: str = "do", latency_us: float = 10.0,
          link_gbs: float = 45.0, links: Optional[int] = None, list_form_edges: int = 1 << 21,
          avg_list_fill: float = 1.0) -> List[dict]:
    """Per-level rows for docs/ARCHITECTURE.md §4: direction, chain form,
    collective launches, MiB sent per rank and an estimate of the exchange
    time: latency_us per launch + bytes over (P - 1) links of link_gbs GB/s
    each (direct exchange over xGMI: each peer on its own link).  Sparse levels
    ship count-sized lists: their bytes here are the frontier edges x 4 B x
    (P - 1) / P (every edge's target an id to its owner, at most),
    avg_list_fill scaling that bound."""
    part = max(64, -(-(-(-n // nranks)) // 64) * 64)
    W = part // 64
    cfg = ModelConfig(nranks=nranks, slice_words=W, mode=mode, fused=True)
    rows = []
    links = links if links is not None else max(1, nranks - 1)
    gathered = mode == "bu"
    for level, form, cap, gather in predicted_forms(levels, cfg, list_form_edges):
        t = chain_traffic(cfg, form, cap, gather, gathered)
        gathered = gather
        mf = levels[level][1] if level < len(levels) else 0
        nbytes = t.total_bytes
        if form == "S":
            # count-sized: the ids actually sent, not the capacity
            nbytes += int(mf * 4 * (nranks - 1) / nranks * avg_list_fill) - (nranks - 1) * (cap + 1) * 4
        mib = nbytes / 2**20
        est = t.total_calls * latency_us + nbytes / (links * link_gbs * 1e3)
        d = levels[level][0] if level < len(levels) else "-"
        rows.append({"level": level, "dir": d, "frontier_edges": mf, "form": form, "gather": gather,
                     "collectives": t.total_calls,
                     "kinds": {k: v for k, v in t.calls.items() if k != "fused"},
                     "mib_per_rank": round(mib, 3), "est_us": round(est, 1)})
    return rows
