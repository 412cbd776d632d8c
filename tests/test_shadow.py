"""Shadow rank: a rank of a P-rank job replayed alone from its recorded
collective outputs (RecordComm -> ReplayComm) reproduces the recorded run."""
import numpy as np
import pytest

import distributed_cuda_bfs_amd as dbfs
from distributed_cuda_bfs_amd.parallel.runtime import make_backend
from distributed_cuda_bfs_amd.parallel.shadow import shadow_ranks

N = dbfs.native


@pytest.mark.parametrize("P,mode", [(2, "do"), (3, "do"), (4, "td"), (4, "bu")])
def test_replay_matches_recorded_run(P, mode):
    p = dbfs.rmat_params(11, 16, 5)
    csr = dbfs.host_csr_from_params(p)
    roots = [3, 77, 500]
    runs = shadow_ranks(p, P, [0, P - 1], roots, mode=mode, device="cpu")
    part = dbfs.native.Partition(p.n, P)
    for s in runs:
        assert s.exact, (s.rank, s.levels, s.recorded_levels)
        assert s.tape_records > 0 and len(s.collectives) > 0
        assert len(s.levels) == len(roots)
        # the replayed rank's level count equals the oracle's depth (one less
        # when every vertex with an edge was reached: the last frontier is not
        # expanded)
        exp = dbfs.cpu_bfs(csr, roots[-1])[0]
        depth = int(exp[exp != dbfs.UNREACHED].max()) + 1
        assert len(s.levels[-1]) in (depth, depth - 1)
    assert part.nranks == P


def test_replay_rejects_a_different_schedule():
    """A replayed rank that issues another collective than the tape's next
    one fails loudly instead of reading the wrong output."""
    p = dbfs.rmat_params(10, 16, 5)
    be = make_backend("cpu")
    group = N.VirtualGroup(1)
    rec = N.record_comm(N.virtual_comm(group, 0, be), be)
    from distributed_cuda_bfs_amd.parallel.runtime import Runtime
    rt = Runtime(backend=be, comm=rec, rank=0, world=1)
    bfs = dbfs.BFS(p, rt, mode="do", force_exchange=True)
    bfs.run(5)
    tape = rec.tape
    assert len(tape) > 0
    rp = N.replay_comm(tape, be)
    rt2 = Runtime(backend=be, comm=rp, rank=0, world=1)
    bfs2 = dbfs.BFS(p, rt2, mode="do", force_exchange=True)
    bfs2.engine.set_option("list_form_edges", 0)  # another exchange schedule than recorded
    with pytest.raises(Exception, match="ReplayComm"):
        bfs2.run(5)
        bfs2.run(5)
    np.testing.assert_equal(rp.position <= len(rp), True)
