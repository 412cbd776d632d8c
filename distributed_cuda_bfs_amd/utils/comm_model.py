"""Per-level communication model of the multi-rank device loop.

Mirrors what ``Engine::run_bitmap_device`` (csrc/engine/engine.cpp,
``enqueue_level`` / ``finish_ranks``) issues for each level chain, so the
collectives and bytes of a traversal can be predicted from its chain forms
(``BFSResult.chains``) and checked against the communicators' traffic
counters (``Comm.traffic()``, tests/test_comm_model.py).  ``table`` turns a
1-GPU level profile into the per-level bytes / collectives table of
docs/ARCHITECTURE.md §4.

Bytes are what one rank sends to the other ranks under a direct exchange:
alltoall / allgather (P - 1) x the per-peer bytes, all-reduce (P - 1) x the
vector, alltoallv the counts to other ranks.

Reference being replaced: the per-level exchange of bfs.cu:587-609 (owner
buckets copied peer to peer after a count exchange) and bfs_mpi.cu:601-621.
"""
from __future__ import annotations

from collections import Counter
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

WORD = 8  # bytes per bitmap word (64 vertices)


@dataclass
class ModelConfig:
    nranks: int
    slice_words: int              # Partition.slice_words(): words of one rank's bitmap slice
    hub_words: int = 0            # ceil(nhubs / 64) (0: no hubs -> no split bottom-up levels)
    mode: str = "do"              # engine mode: do / td / bu
    bu_split: bool = True         # EngineOptions.bu_split (needs hubs)

    @property
    def split_ok(self) -> bool:
        return self.nranks > 1 and self.bu_split and self.hub_words > 0 and self.mode != "td"


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
        return sum(v for k, v in self.calls.items() if k != "barrier")


def chain_traffic(cfg: ModelConfig, form: str, cap: int, in_carry: bool) -> Tuple[ChainTraffic, bool]:
    """Collectives of one level chain; returns (traffic, carry) where carry says
    whether its totals reduction carried the hub frontier bits."""
    P, W = cfg.nranks, cfg.slice_words
    t = ChainTraffic()
    split = form == "B" and cfg.split_ok and in_carry
    if not split and (form == "B" or cfg.mode != "do"):
        t.add("allgather", (P - 1) * W * WORD)             # frontier slices (+ visited merge)
    if form == "L":
        t.add("alltoallv", (P - 1) * (cap + 1) * 4)         # owner lists, count first
    elif form == "T":
        t.add("alltoall", (P - 1) * W * WORD)               # candidate bitmap slices
    elif form == "B" and split:
        t.add("allgather", (P - 1) * W * WORD)              # on the side stream, under the head pass
    carry = cfg.split_ok and form != "L"
    t.add("allreduce", (P - 1) * 8 * (2 + (cfg.hub_words if carry else 0)))  # totals (+ hub bits)
    return t, carry


def run_traffic(cfg: ModelConfig, chains: Iterable[Tuple[int, str, int]]) -> ChainTraffic:
    """Traffic of one traversal from its enqueued chains (level, form, cap):
    start barrier, seed totals, every chain, the wall-time max at the end."""
    P = cfg.nranks
    tot = ChainTraffic()
    tot.add("barrier", 0)
    seed_carry = cfg.split_ok and cfg.mode == "bu"
    tot.add("allreduce", (P - 1) * 8 * (2 + (cfg.hub_words if seed_carry else 0)))
    carry_of: Dict[int, bool] = {-1: seed_carry}
    for level, form, cap in chains:
        t, carry = chain_traffic(cfg, form, int(cap), carry_of.get(level - 1, False))
        carry_of[level] = carry
        tot.merge(t)
    tot.add("allgather", (P - 1) * 8)  # max over ranks of the wall time
    return tot


def list_cap_for(mf: float, list_max: int, factor: float = 4.0) -> int:
    """The engine's list capacity for a predicted frontier of mf edges (0: dense)."""
    if list_max <= 0:
        return 0
    want = max(1024.0, mf * factor)
    if want > list_max:
        return 0
    c = 1024
    while c < want:
        c <<= 1
    return min(c, list_max)


def predicted_forms(levels: Sequence[Tuple[str, int]], cfg: ModelConfig,
                    list_form_edges: int = 1 << 16) -> List[Tuple[int, str, int]]:
    """Chains of a perfectly predicted traversal with per-level (direction,
    frontier edges), plus the trailing no-op chain the loop enqueues ahead."""
    list_max = min(list_form_edges, max(cfg.slice_words, 1024)) if cfg.mode != "bu" else 0
    out = []
    for L, (d, mf) in enumerate(list(levels) + [("T", 0)]):
        if d == "B":
            out.append((L, "B", 0))
        else:
            cap = list_cap_for(mf, list_max)
            out.append((L, "L" if cap else "T", cap))
    return out


def table(levels: Sequence[Tuple[str, int]], n: int, nranks: int, nhubs: int = 1 << 19, mode: str = "do",
          latency_us: float = 10.0, link_gbs: float = 45.0, links: Optional[int] = None) -> List[dict]:
    """Per-level rows for docs/ARCHITECTURE.md §4: direction, chain form,
    collectives, MiB sent per rank and an estimate of the exchange time:
    latency_us per collective + bytes over (P - 1) links of link_gbs GB/s each
    (direct exchange over xGMI: each peer on its own link)."""
    part = max(64, -(-(-(-n // nranks)) // 64) * 64)
    cfg = ModelConfig(nranks=nranks, slice_words=part // 64, hub_words=-(-nhubs // 64), mode=mode)
    rows = []
    carry_prev = cfg.split_ok and mode == "bu"
    links = links if links is not None else max(1, nranks - 1)
    for level, form, cap in predicted_forms(levels, cfg):
        t, carry_prev = chain_traffic(cfg, form, cap, carry_prev)
        mib = t.total_bytes / 2**20
        est = t.total_calls * latency_us + t.total_bytes / (links * link_gbs * 1e3)
        d = levels[level][0] if level < len(levels) else "-"
        mf = levels[level][1] if level < len(levels) else 0
        rows.append({"level": level, "dir": d, "frontier_edges": mf, "form": form, "collectives": t.total_calls,
                     "kinds": dict(t.calls), "mib_per_rank": round(mib, 3), "est_us": round(est, 1)})
    return rows
