"""The per-level communication model (distributed_cuda_bfs_amd/utils/comm_model.py,
docs/ARCHITECTURE.md §4) against the communicators' traffic counters: for every
traversal of virtual ranks on the CPU backend the collectives and bytes each
rank issued equal the model's prediction from the chains the device loop
enqueued (mispredicted and trailing chains included)."""
import numpy as np
import pytest

import distributed_cuda_bfs_amd as dbfs
from distributed_cuda_bfs_amd.parallel.runtime import run_virtual_ranks
from distributed_cuda_bfs_amd.utils.comm_model import ModelConfig, run_traffic, table


@pytest.mark.parametrize("P", [2, 3, 4])
@pytest.mark.parametrize("mode", ["do", "td", "bu"])
@pytest.mark.parametrize("knobs", [{}, {"list_form_edges": 0}, {"list_form_edges": 64}])
def test_traffic_matches_model(P, mode, knobs):
    p = dbfs.rmat_params(12, 16, 17)

    def body(rt):
        b = dbfs.BFS(p, rt, mode=mode)
        for k, v in knobs.items():
            b.engine.set_option(k, v)
        out = []
        for src in (3, 1500, 77):
            b.run(src)  # warm-up (one-time degree moments)
            rt.comm.reset_traffic()
            r = b.run(src)
            out.append((r.chains, rt.comm.traffic()))
        return out, b.partition.slice_words()

    for outs, W in run_virtual_ranks(P, body, device="cpu"):
        cfg = ModelConfig(nranks=P, slice_words=W, mode=mode, list_form_edges=knobs.get("list_form_edges", 1 << 21))
        for chains, got in outs:
            want = run_traffic(cfg, chains)
            for kind, (calls, nbytes) in got.items():
                assert calls == want.calls[kind], (kind, chains, got, dict(want.calls))
                assert nbytes == want.bytes[kind], (kind, chains, got, dict(want.bytes))
            # one collective per chain (its level's end), plus a top-down
            # (or hub-cut) chain's payload exchange; a bottom-up chain's input frontier came
            # with the previous collective unless that one mispredicted; none
            # for the seed (every rank seeds itself), one wall-time max
            fused = run_traffic(ModelConfig(nranks=P, slice_words=W, mode=mode, fused=True,
                                            list_form_edges=cfg.list_form_edges), chains)
            n_td = sum(1 for c in chains if c[1] in "ST")

            def gathered_before(i):
                # the previous level's collective (its last chain: a
                # mispredicted chain of this level in between does not count)
                lv = chains[i][0]
                prev = [c for c in chains[:i] if c[0] == lv - 1]
                return prev[-1][3] if prev else mode == "bu"

            n_lone_b = sum(1 for i, c in enumerate(chains) if c[1] == "B" and not gathered_before(i))
            # (a hub-cut bottom-up chain: its remote claims' all-to-all)
            n_cut = sum(1 for c in chains if c[1] == "B" and c[7])
            assert fused.total_calls == len(chains) + n_td + n_lone_b + n_cut + 1


def test_table_shapes():
    levels = [("T", 5), ("T", 547726), ("B", 911126127), ("B", 1226480949), ("B", 9282057), ("T", 25207),
              ("T", 75)]
    rows = table(levels, 1 << 26, 8)
    assert [r["form"] for r in rows] == ["S", "S", "B", "B", "B", "S", "S", "S"]
    # the level before a bottom-up one gathers its frontier in its collective
    assert [r["gather"] for r in rows] == [False, True, True, True, False, False, False, False]
    # sparse top-down levels: the owner lists, then the totals (+ frontier) in one launch
    assert rows[1]["kinds"] == {"alltoallv": 1, "allgather": 1, "allreduce": 1}
    assert rows[1]["collectives"] == 2
    # bottom-up levels: ONE collective each (their input came with the previous one)
    assert all(r["collectives"] == 1 for r in rows[2:5])
    assert rows[2]["mib_per_rank"] == pytest.approx((7 * (1 << 26) / 8 / 8 + 7 * 16) / 2**20, rel=0.01)
    # sparse levels ship count-sized lists: far below a bitmap slice
    assert rows[5]["mib_per_rank"] < 0.2
    assert sum(r["collectives"] for r in rows) <= len(rows) + 5
    assert all(np.isfinite(r["est_us"]) for r in rows)
