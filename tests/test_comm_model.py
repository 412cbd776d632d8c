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
@pytest.mark.parametrize("knobs", [{}, {"bu_split": 0}, {"list_form_edges": 0}])
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
        return out, b.partition.slice_words(), b.graph.nhubs

    for outs, W, nhubs in run_virtual_ranks(P, body, device="cpu"):
        cfg = ModelConfig(nranks=P, slice_words=W, hub_words=-(-nhubs // 64), mode=mode,
                          bu_split=knobs.get("bu_split", 1) != 0)
        for chains, got in outs:
            want = run_traffic(cfg, chains)
            for kind, (calls, nbytes) in got.items():
                assert calls == want.calls[kind], (kind, chains, got, dict(want.calls))
                assert nbytes == want.bytes[kind], (kind, chains, got, dict(want.bytes))


def test_table_shapes():
    levels = [("T", 5), ("T", 547726), ("B", 911126127), ("B", 1226480949), ("B", 9282057), ("T", 25207),
              ("T", 75)]
    rows = table(levels, 1 << 26, 8)
    assert [r["form"] for r in rows] == ["L", "T", "B", "B", "B", "T", "L", "L"]
    # a dense top-down level ships (P - 1) / P of an N-bit bitmap per rank,
    # plus the totals all-reduce carrying the 2^19 hub frontier bits
    assert rows[1]["mib_per_rank"] == pytest.approx((7 * (1 << 26) / 8 / 8 + 7 * 8 * (2 + 8192)) / 2**20, rel=0.01)
    assert rows[1]["kinds"] == {"alltoall": 1, "allreduce": 1}
    assert rows[2]["kinds"] == {"allgather": 1, "allreduce": 1}
    assert all(np.isfinite(r["est_us"]) for r in rows)
