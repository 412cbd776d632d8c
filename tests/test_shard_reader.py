"""Sharded file ingestion (csrc/graph/shard_reader.cpp, DeviceGraph::from_edges /
from_file): every rank parses only its byte range of the edge list and the CSR
shard is built on its device from owner-routed entries.

Replaces the reference's whole-file read on every rank (bfs.cu:829-880 run by
each MPI rank at bfs_mpi.cu:815).  Virtual ranks on the CPU backend run the
same collective code path as GPU ranks (the kernels differ only in their
bodies).
"""
import os

import numpy as np
import pytest

import distributed_cuda_bfs_amd as dbfs
from distributed_cuda_bfs_amd.parallel.runtime import run_virtual_ranks

N = dbfs.native


def _edges(n, m, seed):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, n, m, dtype=np.int64)
    v = rng.integers(0, n, m, dtype=np.int64)
    return u, v


def _write_ref(path, n, u, v, layout="lines", tail=""):
    toks = []
    for a, b in zip(u.tolist(), v.tolist()):
        toks.append((a, b))
    with open(path, "w") as f:
        f.write(f"{n} {len(toks)}\n")
        if layout == "lines":
            f.write("".join(f"{a} {b}\n" for a, b in toks))
        elif layout == "split":  # pairs straddle lines, uneven spacing
            flat = [x for ab in toks for x in ab]
            for i, x in enumerate(flat):
                f.write(str(x) + ("\n" if i % 3 == 2 else "  \t"))
        elif layout == "wide":  # several pairs per line
            for i in range(0, len(toks), 5):
                f.write(" ".join(f"{a} {b}" for a, b in toks[i:i + 5]) + "\r\n")
        f.write(tail)


def _shards(path, P, threads=0):
    def body(rt):
        s = N.read_edge_shard(path, rt.comm, threads)
        return (s.n, s.m, s.first_edge, s.byte_begin, s.byte_end, np.asarray(s.u).copy(), np.asarray(s.v).copy())

    return run_virtual_ranks(P, body, device="cpu")


@pytest.mark.parametrize("layout", ["lines", "split", "wide"])
@pytest.mark.parametrize("P", [1, 2, 3, 5])
def test_ranks_read_disjoint_byte_ranges(tmp_path, layout, P):
    n, m = 1000, 4000
    u, v = _edges(n, m, 3)
    path = str(tmp_path / "g.txt")
    _write_ref(path, n, u, v, layout)
    size = os.path.getsize(path)
    outs = _shards(path, P, threads=4)
    # byte ranges: disjoint, in rank order, covering the body, about size / P each
    begins = [o[3] for o in outs]
    ends = [o[4] for o in outs]
    assert ends[-1] == size
    for r in range(1, P):
        assert begins[r] == ends[r - 1]
    for o in outs:
        assert o[4] - o[3] <= size // P + 64
    # edges: the file's edges in order, each exactly once
    got_u = np.concatenate([o[5] for o in outs])
    got_v = np.concatenate([o[6] for o in outs])
    assert np.array_equal(got_u, u) and np.array_equal(got_v, v)
    assert [o[2] for o in outs] == list(np.cumsum([0] + [len(o[5]) for o in outs[:-1]]))
    assert all(o[0] == n and o[1] == m for o in outs)


def test_trailing_tokens_ignored_and_threads(tmp_path):
    n, m = 500, 3001
    u, v = _edges(n, m, 4)
    path = str(tmp_path / "g.txt")
    _write_ref(path, n, u, v, "split", tail="7 8 9 garbage\n")
    for P in (1, 3):
        for threads in (1, 3, 8):
            outs = _shards(path, P, threads)
            assert np.array_equal(np.concatenate([o[5] for o in outs]), u)
            assert np.array_equal(np.concatenate([o[6] for o in outs]), v)


@pytest.mark.parametrize("P", [1, 3])
def test_errors_agree_on_every_rank(tmp_path, P):
    path = str(tmp_path / "bad.txt")
    with open(path, "w") as f:
        f.write("10 4\n0 1\n2 3\n4 5\n")  # truncated
    with pytest.raises(Exception, match="truncated"):
        _shards(path, P)
    with open(path, "w") as f:
        f.write("10 3\n0 1\n2 11\n4 5\n")  # out of range
    with pytest.raises(Exception, match="out of range"):
        _shards(path, P)
    with open(path, "w") as f:
        f.write("10 2\n0 1\n2 3x\n")  # malformed token used by an edge
    with pytest.raises(Exception, match="out of range|malformed"):
        _shards(path, P)


def test_matrix_market_shards(tmp_path):
    n, m = 300, 2000
    u, v = _edges(n, m, 5)
    path = str(tmp_path / "g.mtx")
    with open(path, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n% a comment\n%\n")
        f.write(f"{n} {n} {m}\n")
        for i, (a, b) in enumerate(zip(u.tolist(), v.tolist())):
            if i % 97 == 0:
                f.write("% interleaved comment\n")
            f.write(f"{a + 1} {b + 1} {0.5 * i:.3f}\n")
    for P in (1, 2, 4):
        outs = _shards(path, P, threads=3)
        assert np.array_equal(np.concatenate([o[5] for o in outs]), u)
        assert np.array_equal(np.concatenate([o[6] for o in outs]), v)


def _row_multisets(csr_rows_off, col, lo, hi, full_off, full_col):
    for r in range(lo, hi):
        a = np.sort(col[csr_rows_off[r - lo]:csr_rows_off[r - lo + 1]])
        b = np.sort(full_col[full_off[r]:full_off[r + 1]])
        assert np.array_equal(a, b), r


@pytest.mark.parametrize("P", [1, 3, 4])
def test_device_shards_match_full_csr(tmp_path, P):
    n, m = 777, 5000
    u, v = _edges(n, m, 6)
    path = str(tmp_path / "g.txt")
    _write_ref(path, n, u, v, "wide")
    full = dbfs.read_graph(path)
    fo, fc = np.asarray(full.row_off), np.asarray(full.col)

    def body(rt):
        g = N.DeviceGraph.from_file(rt.backend, rt.comm, path, 2)
        h = g.to_host()
        return g.lo, g.rows, g.input_edges, np.asarray(h.row_off).copy(), np.asarray(h.col).copy()

    outs = run_virtual_ranks(P, body, device="cpu")
    assert sum(o[1] for o in outs) == n
    for lo, rows, me, ro, col in outs:
        assert me == m
        _row_multisets(ro, col, lo, lo + rows, fo, fc)


@pytest.mark.parametrize("mode", ["do", "td", "ref"])
def test_bfs_on_sharded_load_matches_oracle(tmp_path, mode):
    p = dbfs.rmat_params(11, 8, 13)
    csr = dbfs.host_csr_from_params(p)
    # write the generator's edges as a reference-format file
    u, v = (np.asarray(x, dtype=np.int64) for x in dbfs.generate_edges(p))
    path = str(tmp_path / "rmat.txt")
    _write_ref(path, p.n, u, v, "lines")
    srcs = [0, 17, 1000]
    exp = [dbfs.cpu_bfs(csr, s)[0] for s in srcs]

    def body(rt):
        b = dbfs.BFS(path, rt, mode=mode)
        out = []
        for s in srcs:
            b.run(s)
            out.append(b.levels())
        return out

    for rank_out in run_virtual_ranks(3, body, device="cpu"):
        for got, e in zip(rank_out, exp):
            assert np.array_equal(got, e)


def test_binary_cache_sharded_rows(tmp_path):
    p = dbfs.rmat_params(10, 8, 2)
    csr = dbfs.host_csr_from_params(p)
    path = str(tmp_path / "g.csr")
    dbfs.write_binary_csr(path, csr)
    fo, fc = np.asarray(csr.row_off), np.asarray(csr.col)

    def body(rt):
        g = N.DeviceGraph.from_file(rt.backend, rt.comm, path)
        h = g.to_host()
        return g.lo, g.rows, np.asarray(h.row_off).copy(), np.asarray(h.col).copy()

    for lo, rows, ro, col in run_virtual_ranks(3, body, device="cpu"):
        assert np.array_equal(ro, fo[lo:lo + rows + 1] - fo[lo])
        assert np.array_equal(col, fc[fo[lo]:fo[lo + rows]])
