"""Graph ingestion, CSR construction, generators and the CPU oracle (CPU only).

Reference behaviour pinned here: readGraphFromFile (bfs.cu:829-880) symmetrises
every input edge in file order, keeps duplicates and self-loops (a self-loop
appears twice), numEdges = 2m; bfsCPU (bfs.cu:923-945) gives the exact levels.
"""
import os

import numpy as np
import pytest

import distributed_cuda_bfs_amd as dbfs
from distributed_cuda_bfs_amd.utils.validate import check_levels_against_oracle, levels_are_consistent

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

U = dbfs.UNREACHED


def test_chain8_levels(data_dir):
    csr = dbfs.read_graph(os.path.join(data_dir, "chain8.txt"))
    assert csr.n == 8 and csr.input_edges == 7 and csr.directed_edges == 14
    lv, par = dbfs.cpu_bfs(csr, 0)
    assert lv.tolist() == list(range(8))
    assert par[0] == -1


def test_reference_adjacency_order(data_dir):
    csr = dbfs.read_graph(os.path.join(data_dir, "two_components.txt"))
    ro, col = np.asarray(csr.row_off), np.asarray(csr.col)
    # adj[u] += v ; adj[v] += u per input edge in file order (bfs.cu:860-861)
    assert col[ro[0]:ro[1]].tolist() == [1, 0 + 2]  # edges (0,1) then (2,0)
    assert col[ro[2]:ro[3]].tolist() == [1, 0]
    assert col[ro[5]:ro[6]].tolist() == [4, 5, 5]  # self-loop appears twice
    assert csr.directed_edges == 14


def test_two_components_unreached(data_dir):
    csr = dbfs.read_graph(os.path.join(data_dir, "two_components.txt"))
    lv, _ = dbfs.cpu_bfs(csr, 3)
    assert lv.tolist() == [U, U, U, 0, 1, 2, U, U, U, U]
    assert levels_are_consistent(csr, lv, 3)


def test_matrix_market(data_dir):
    p = os.path.join(data_dir, "dup_self.mtx")
    assert dbfs.detect_format(p) == "mtx"
    n, u, v = dbfs.read_edge_list(p)
    assert n == 7 and len(u) == 9
    assert (u[0], v[0]) == (0, 1)  # 1-based -> 0-based
    csr = dbfs.read_graph(p)
    lv, _ = dbfs.cpu_bfs(csr, 0)
    assert lv.tolist() == [0, 1, 2, 3, 3, 2, 1]


def test_bad_inputs(tmp_path):
    bad = tmp_path / "bad.txt"
    bad.write_text("3 2\n0 1\n1 7\n")
    with pytest.raises(RuntimeError, match="out of range"):
        dbfs.read_graph(str(bad))
    trunc = tmp_path / "trunc.txt"
    trunc.write_text("3 5\n0 1\n")
    with pytest.raises(RuntimeError, match="truncated"):
        dbfs.read_graph(str(trunc))
    with pytest.raises(RuntimeError, match="not open"):
        dbfs.read_graph(str(tmp_path / "missing.txt"))


def test_binary_cache_roundtrip(tmp_path):
    p = dbfs.rmat_params(10, 8, 4)
    csr = dbfs.host_csr_from_params(p)
    f = str(tmp_path / "g.csr")
    dbfs.ops.write_binary_csr(f, csr)
    assert dbfs.detect_format(f) == "binary"
    back = dbfs.read_graph(f)
    assert np.array_equal(np.asarray(back.row_off), np.asarray(csr.row_off))
    assert np.array_equal(np.asarray(back.col), np.asarray(csr.col))
    assert back.input_edges == csr.input_edges


def test_binary_cache_shard_reads(tmp_path):
    """Version-2 cache: a rank reads only its rows (rebased offsets, global
    column ids) and the shards concatenate to the whole graph."""
    p = dbfs.rmat_params(12, 8, 5)
    csr = dbfs.host_csr_from_params(p)
    f = str(tmp_path / "g.csr")
    dbfs.ops.write_binary_csr(f, csr)
    info = dbfs.native.binary_csr_info(f)
    assert info["version"] == 2 and info["n"] == csr.n and info["nnz"] == csr.directed_edges
    ro, col = np.asarray(csr.row_off), np.asarray(csr.col)
    part = dbfs.native.Partition(csr.n, 3)
    cols = []
    for r in range(3):
        lo, hi = part.lo(r), part.hi(r)
        sh = dbfs.native.read_binary_csr_rows(f, lo, hi)
        assert sh.row_lo == lo and sh.rows == hi - lo and sh.n == csr.n
        assert np.array_equal(np.asarray(sh.row_off), ro[lo:hi + 1] - ro[lo])
        cols.append(np.asarray(sh.col))
    assert np.array_equal(np.concatenate(cols), col)
    with pytest.raises(RuntimeError, match="outside"):
        dbfs.native.read_binary_csr_rows(f, 0, csr.n + 1)


def _corrupt(src, dst, offset, data):
    b = bytearray(open(src, "rb").read())
    if offset is None:
        b = b[:data]
    else:
        b[offset:offset + len(data)] = data
    open(dst, "wb").write(bytes(b))


def test_binary_cache_rejects_corruption(tmp_path):
    """Truncated or corrupted caches raise instead of handing out-of-range ids
    or offsets to the device (header trusted, col unchecked)."""
    import struct
    p = dbfs.rmat_params(10, 8, 4)
    csr = dbfs.host_csr_from_params(p)
    f = str(tmp_path / "g.csr")
    dbfs.ops.write_binary_csr(f, csr)
    hdr = 8 + 4 + 4 + 5 * 8 + 2 * 8 + 8
    n_off = (csr.rows + 1) * 8
    cases = {
        "trunc": (None, hdr + 10),
        "trunc_cols": (None, hdr + n_off + 16),
        "header_rows": (16 + 16, struct.pack("<q", -5)),          # rows field (header checksum)
        "header_nnz_huge": (16 + 24, struct.pack("<q", 1 << 62)),  # nnz field
        "row_off": (hdr + 8 * 5, struct.pack("<q", 1 << 40)),      # an offset (block checksum)
        "col": (hdr + n_off + 4 * 7, struct.pack("<I", 0xFFFFFFF0)),  # a column id
    }
    for name, (off, data) in cases.items():
        g = str(tmp_path / f"{name}.csr")
        _corrupt(f, g, off, data)
        with pytest.raises(RuntimeError):
            dbfs.read_graph(g)


def test_binary_cache_v1_structural_checks(tmp_path):
    """Round-1 (version 1) caches are still read, with the structural checks:
    a column id >= n is rejected even though v1 checksums only the offsets."""
    import struct
    p = dbfs.rmat_params(9, 8, 3)
    csr = dbfs.host_csr_from_params(p)
    ro = np.asarray(csr.row_off, dtype=np.int64)
    col = np.asarray(csr.col, dtype=np.uint32).copy()

    def fnv(b):
        h = 1469598103934665603
        for x in b:
            h = ((h ^ x) * 1099511628211) & (2 ** 64 - 1)
        return h

    def write(path, col_arr):
        hdr = b"DBFSCSR1" + struct.pack("<II", 1, 0) + struct.pack(
            "<qqqqq", csr.n, 0, csr.rows, csr.directed_edges, csr.input_edges) + struct.pack("<Q", fnv(ro.tobytes()))
        open(path, "wb").write(hdr + ro.tobytes() + col_arr.tobytes())

    good = str(tmp_path / "v1.csr")
    write(good, col)
    back = dbfs.read_graph(good)
    assert np.array_equal(np.asarray(back.col), col)
    col[3] = csr.n + 7
    bad = str(tmp_path / "v1bad.csr")
    write(bad, col)
    with pytest.raises(RuntimeError, match="column id"):
        dbfs.read_graph(bad)


def test_levels_out_format(tmp_path):
    f = str(tmp_path / "l.txt")
    dbfs.ops.write_levels(f, np.array([0, 1, U], dtype=np.int32))
    assert open(f).read() == "0\n1\n2147483647\n"


def test_generator_deterministic_and_scrambled():
    p = dbfs.rmat_params(14, 16, 1)
    u1, v1 = dbfs.generate_edges(p, 0, 1000)
    u2, v2 = dbfs.generate_edges(p, 500, 1000)
    assert np.array_equal(u1[500:], u2) and np.array_equal(v1[500:], v2)
    assert u1.max() < p.n and v1.max() < p.n
    # scramble spreads the hubs: vertex 0 is not the top-degree vertex
    u, v = dbfs.generate_edges(p)
    deg = np.bincount(np.concatenate([u, v]), minlength=p.n)
    assert deg.sum() == 2 * p.m
    assert int(np.argmax(deg)) != 0
    # a different seed gives a different graph
    q = dbfs.rmat_params(14, 16, 2)
    u3, _ = dbfs.generate_edges(q, 0, 1000)
    assert not np.array_equal(u1, u3)


def test_scramble_is_bijective():
    N = dbfs.native
    for scale in (1, 5, 10):
        xs = [N.scramble_vertex(x, scale, 42) for x in range(1 << scale)]
        assert sorted(xs) == list(range(1 << scale))


def test_rmat_skew():
    p = dbfs.rmat_params(12, 16, 3)
    u, v = dbfs.generate_edges(p)
    deg = np.bincount(np.concatenate([u, v]), minlength=p.n)
    assert deg.max() > 20 * deg.mean()  # power-law hubs


def test_uniform_generator():
    p = dbfs.uniform_params(1000, 5000, 3)
    u, v = dbfs.generate_edges(p)
    assert len(u) == 5000 and u.max() < 1000 and v.max() < 1000


def test_check_levels_against_oracle():
    assert check_levels_against_oracle([0, 1, 2], [0, 1, 2]) is None
    assert check_levels_against_oracle([0, 2, 2], [0, 1, 2]) == (1, 2, 1)


def test_partition_block_rounding():
    N = dbfs.native
    p = N.Partition(1000, 3)
    assert p.part % 64 == 0 and p.part * 3 >= 1000
    owners = [p.owner(v) for v in range(1000)]
    assert min(owners) == 0 and max(owners) == 2
    assert sum(p.count(r) for r in range(3)) == 1000
    assert p.lo(0) == 0 and p.hi(2) == 1000
    # N % P != 0 with tiny N: every vertex still has a valid owner (reference defect D5)
    q = N.Partition(5, 4)
    assert all(0 <= q.owner(v) < 4 for v in range(5))
    assert sum(q.count(r) for r in range(4)) == 5


def test_directed_stdin_reader_and_engine(tmp_path):
    # the reference's stdin reader (readGraph, bfs.cu:882-920): pairs as
    # directed edges, no symmetrisation; top-down modes on the CSR of out-edges
    import subprocess
    import sys

    import distributed_cuda_bfs_amd as dbfs
    from distributed_cuda_bfs_amd.parallel.runtime import init_runtime

    text = "6 5\n0 1\n1 2\n3 2\n2 4\n4 0\n"
    path = tmp_path / "d.txt"
    path.write_text(text)
    g = dbfs.read_graph(str(path), directed=True)
    assert g.directed_edges == 5 and np.diff(np.asarray(g.row_off)).tolist() == [1, 1, 1, 1, 1, 0]
    exp, _ = dbfs.cpu_bfs(g, 0)
    assert exp.tolist() == [0, 1, 2, dbfs.UNREACHED, 3, dbfs.UNREACHED]
    rt = init_runtime("cpu")
    for mode in ("td", "ref", "simple", "scan"):
        for P in (1,):
            bfs = dbfs.BFS(g, rt, mode=mode, directed=True)
            res = bfs.run(0)
            assert np.array_equal(bfs.levels(), exp), mode
            assert res.reached == 4 and res.edges == 4, (mode, res.reached, res.edges)
    with pytest.raises(ValueError):
        dbfs.BFS(g, rt, mode="do", directed=True)
    # CLI, edge list on standard input
    out = subprocess.run([os.path.join(REPO, "bin", "bfs"), "0", "-", "--cpu", "--directed", "--quiet",
                          "--levels-out", str(tmp_path / "lv.txt")], input=text, capture_output=True, text=True,
                         timeout=60)
    assert out.returncode == 0, out.stderr
    assert (tmp_path / "lv.txt").read_text().split() == ["0", "1", "2", "2147483647", "3", "2147483647"]


def test_python_partition_vectorised_matches_native():
    """The numpy forms of Partition (owners / to_local / to_global / route /
    split / assemble) agree with the native per-vertex answers, including an
    N that P does not divide (reference defect D5: no out-of-range owner)."""
    import numpy as np
    for n, p in [(1000, 3), (4847571, 8), (5, 4), (64, 1)]:
        part = dbfs.Partition(n, p)
        v = np.unique(np.concatenate([np.arange(min(n, 200)), np.linspace(0, n - 1, 200).astype(np.int64)]))
        own = part.owners(v)
        assert own.max() < p
        assert all(int(o) == part.owner(int(x)) for o, x in zip(own, v))
        loc = part.to_local(v)
        assert all(int(part.to_global(int(o), [int(l)])[0]) == int(x) for o, l, x in zip(own, loc, v))
        buckets = part.route(v[::-1])
        assert sum(len(b) for b in buckets) == len(v)
        for r, b in enumerate(buckets):
            assert all(part.owner(int(x)) == r for x in b)
            assert list(b) == sorted(b, reverse=True)  # input order kept
        if n <= 5000:
            full = np.arange(n) * 3
            assert np.array_equal(part.assemble(part.split(full)), full)
    with pytest.raises(ValueError):
        dbfs.Partition(10, 2).owners([10])
