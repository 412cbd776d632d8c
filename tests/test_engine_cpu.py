"""Engine orchestration on the CPU backend (same C++ engine the GPU runs).

Covers every mode, the direction-optimising switch, P virtual ranks with N not
divisible by P (reference defect D5), isolated / last-vertex sources, and the
device-side Graph500 validation.
"""
import numpy as np
import pytest

import distributed_cuda_bfs_amd as dbfs
from distributed_cuda_bfs_amd.parallel.runtime import init_runtime, run_virtual_ranks

MODES = list(dbfs.MODES)


@pytest.fixture(scope="module")
def rt():
    return init_runtime("cpu")


def _oracle(csr, src):
    return dbfs.cpu_bfs(csr, src)[0]


@pytest.mark.parametrize("mode", MODES)
def test_modes_match_oracle(rt, mode):
    p = dbfs.rmat_params(11, 16, 7)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, rt, mode=mode)
    for src in bfs.sample_roots(4, seed=1):
        res = bfs.run(src)
        exp = _oracle(csr, src)
        assert np.array_equal(bfs.levels(), exp)
        deg = np.diff(np.asarray(csr.row_off))
        assert res.reached == int((exp != dbfs.UNREACHED).sum())
        assert res.edges == int(deg[exp != dbfs.UNREACHED].sum()) // 2
        assert res.depth == int(exp[exp != dbfs.UNREACHED].max()) + 1
        assert bfs.validate(src)


def test_direction_switches(rt):
    p = dbfs.rmat_params(12, 16, 3)
    bfs = dbfs.BFS(p, rt, mode="do")
    src = bfs.sample_roots(1, seed=5)[0]
    res = bfs.run(src)
    dirs = "".join(l["dir"] for l in res.levels)
    assert "T" in dirs and "B" in dirs, dirs
    assert dirs[0] == "T"


def test_heuristic_extremes_still_exact(rt):
    p = dbfs.rmat_params(11, 16, 9)
    csr = dbfs.host_csr_from_params(p)
    for alpha, beta in [(1e9, 1e9), (1e-9, 1e-9), (2.0, 2.0)]:
        bfs = dbfs.BFS(p, rt, mode="do", alpha=alpha, beta=beta, bu_lane_limit=1)
        bfs.run(17)
        assert np.array_equal(bfs.levels(), _oracle(csr, 17))


def test_isolated_and_last_source(rt):
    p = dbfs.uniform_params(3001, 2000, 5)  # many isolated vertices, odd n
    csr = dbfs.host_csr_from_params(p)
    deg = np.diff(np.asarray(csr.row_off))
    iso = int(np.nonzero(deg == 0)[0][0])
    for mode in MODES:
        bfs = dbfs.BFS(csr, rt, mode=mode)
        for src in (iso, csr.n - 1, 0):
            res = bfs.run(src)
            assert np.array_equal(bfs.levels(), _oracle(csr, src))
        res = bfs.run(iso)
        assert res.reached == 1 and res.edges == 0 and res.depth == 1


def test_self_loops_and_duplicates(rt, data_dir):
    csr = dbfs.read_graph(f"{data_dir}/dup_self.mtx")
    for mode in MODES:
        bfs = dbfs.BFS(csr, rt, mode=mode)
        bfs.run(2)
        assert np.array_equal(bfs.levels(), _oracle(csr, 2))


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("mode", MODES)
def test_virtual_ranks(P, mode):
    p = dbfs.rmat_params(10, 16, 13)
    csr = dbfs.host_csr_from_params(p)
    srcs = [3, 1000, 1023]
    exp = [_oracle(csr, s) for s in srcs]

    def body(rt):
        bfs = dbfs.BFS(csr, rt, mode=mode)
        out = []
        for s in srcs:
            r = bfs.run(s)
            out.append((bfs.levels(), r.reached, r.edges, bfs.validate(s)))
        return out

    for rank_out in run_virtual_ranks(P, body, device="cpu"):
        for (lv, reached, edges, ok), e in zip(rank_out, exp):
            assert np.array_equal(lv, e)
            assert reached == int((e != dbfs.UNREACHED).sum())
            assert ok


def test_virtual_ranks_odd_n_generated_shards():
    # generated shards (device generator path) with N % P != 0 via uniform graph
    p = dbfs.uniform_params(777, 3000, 21)
    csr = dbfs.host_csr_from_params(p)
    exp = _oracle(csr, 776)

    def body(rt):
        bfs = dbfs.BFS(p, rt, mode="do")
        bfs.run(776)
        return bfs.levels(), bfs.local_levels(), bfs.graph.lo, bfs.graph.rows

    outs = run_virtual_ranks(5, body, device="cpu")
    total_rows = 0
    for lv, loc, lo, rows in outs:
        assert np.array_equal(lv, exp)
        assert np.array_equal(loc, exp[lo:lo + rows])
        total_rows += rows
    assert total_rows == 777


def test_mode_switch_on_same_engine(rt):
    p = dbfs.rmat_params(10, 16, 2)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, rt, mode="ref")
    for m in MODES:
        bfs.mode = m
        assert bfs.mode == m
        bfs.run(9)
        assert np.array_equal(bfs.levels(), _oracle(csr, 9))


@pytest.mark.parametrize("mode", MODES)
def test_parent_tree(rt, mode):
    from distributed_cuda_bfs_amd.utils.validate import parents_are_valid

    p = dbfs.rmat_params(10, 8, 4)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, rt, mode=mode)
    src = bfs.sample_roots(1, seed=2)[0]
    bfs.run(src)
    assert parents_are_valid(csr, bfs.levels(), bfs.parents(src), src)


def test_parent_tree_virtual_ranks():
    from distributed_cuda_bfs_amd.utils.validate import parents_are_valid

    p = dbfs.rmat_params(9, 8, 6)
    csr = dbfs.host_csr_from_params(p)

    def body(rt):
        bfs = dbfs.BFS(p, rt, mode="do")
        bfs.run(1)
        return bfs.levels(), bfs.parents(1)

    for lv, par in run_virtual_ranks(3, body, device="cpu"):
        assert parents_are_valid(csr, lv, par, 1)


@pytest.mark.parametrize("cut", [0, 1])
@pytest.mark.parametrize("mode", MODES)
def test_force_exchange_single_rank(rt, mode, cut):
    # the multi-rank exchange path (alltoall / allgather / alltoallv) with P = 1
    # (cut: hub-cut bottom-up levels forced -- the one-rank cut, no owner lists)
    p = dbfs.rmat_params(10, 16, 17)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, rt, mode=mode, force_exchange=True)
    if cut:
        bfs.engine.set_option("bu_cut_edges", 1 << 40)
        bfs.engine.set_option("bu_cut_mf_frac", 1.0)
    for src in bfs.sample_roots(2, seed=3):
        bfs.run(src)
        assert np.array_equal(bfs.levels(), _oracle(csr, src))


@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("mode", ["td", "do"])
def test_td_byte_map_mode(P, mode):
    # td_byte_edges = 0: every top-down level uses the byte map (+ pack for P > 1)
    p = dbfs.rmat_params(11, 16, 29)
    csr = dbfs.host_csr_from_params(p)
    srcs = [0, 5, 2047]
    exp = [_oracle(csr, s) for s in srcs]

    def body(rt):
        bfs = dbfs.BFS(p, rt, mode=mode)
        bfs.engine.set_heuristics(24.0, 24.0, 8, td_byte_edges=0)
        assert bfs.engine.td_byte_edges == 0
        out = []
        for s in srcs:
            bfs.run(s)
            out.append(bfs.levels())
        return out

    for rank_out in run_virtual_ranks(P, body, device="cpu"):
        for lv, e in zip(rank_out, exp):
            assert np.array_equal(lv, e)


@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("mode", ["td", "do"])
@pytest.mark.parametrize("sparse_max", [0, 64, 1 << 40])
def test_sparse_list_exchange(P, mode, sparse_max):
    # sparse_max_edges decides which top-down levels use the owner-list exchange
    p = dbfs.rmat_params(11, 16, 31)
    csr = dbfs.host_csr_from_params(p)
    srcs = [1, 7, 2000]
    exp = [_oracle(csr, s) for s in srcs]

    def body(rt):
        bfs = dbfs.BFS(p, rt, mode=mode)
        bfs.engine.set_heuristics(24.0, 24.0, 8, sparse_max_edges=sparse_max, sparse_size_check=0)
        out = []
        for s in srcs:
            bfs.run(s)
            out.append(bfs.levels())
        return out

    for rank_out in run_virtual_ranks(P, body, device="cpu"):
        for lv, e in zip(rank_out, exp):
            assert np.array_equal(lv, e)


def test_hub_sort_orders_rows_and_keeps_levels(rt):
    p = dbfs.rmat_params(11, 16, 12)
    csr = dbfs.host_csr_from_params(p)
    exp = _oracle(csr, 4)
    bfs = dbfs.BFS(p, rt, mode="do", hub_sort=True, id_order=False)
    assert bfs.graph.hub_sorted and not bfs.graph.col_by_id
    g = bfs.graph.to_host()
    ro, col = np.asarray(g.row_off), np.asarray(g.col)
    deg = np.diff(np.asarray(csr.row_off))
    for r in range(0, g.rows, 37):
        row = col[ro[r]:ro[r + 1]]
        if 2 <= len(row) <= 4096:
            keys = list(zip(-deg[row], row))
            assert keys == sorted(keys)
        # same multiset as the unsorted CSR
        assert sorted(row.tolist()) == sorted(np.asarray(csr.col)[ro[r]:ro[r + 1]].tolist())
    bfs.run(4)
    assert np.array_equal(bfs.levels(), exp)


def test_id_order_top_down_copy_keeps_levels(rt):
    """With hubs, `col` is put in neighbour-id order for the top-down sweeps
    (bottom-up scans the hub-first, hub-encoded copy): every row sorted, same
    multiset, levels unchanged in every mode and loop."""
    p = dbfs.rmat_params(11, 16, 14)
    csr = dbfs.host_csr_from_params(p)
    # no hub selected (cap 0): the hub-free bottom-up kernels scan `col`
    # head-first, so it keeps its order
    assert not dbfs.BFS(p, rt, mode="do", max_hubs=0).graph.col_by_id
    bfs = dbfs.BFS(p, rt, mode="do")
    assert bfs.graph.col_by_id and bfs.graph.nhubs > 0
    g = bfs.graph.to_host()
    ro, col = np.asarray(g.row_off), np.asarray(g.col)
    for r in range(g.rows):
        row = col[ro[r]:ro[r + 1]]
        assert np.all(row[:-1] <= row[1:])
        assert np.array_equal(row, np.sort(np.asarray(csr.col)[ro[r]:ro[r + 1]]))
    for mode in ("do", "td", "bu"):
        bfs.mode = mode
        for opt in ({}, {"device_loop": 0}):
            for k, v in opt.items():
                bfs.engine.set_option(k, v)
            for s in (4, 77):
                bfs.run(s)
                assert np.array_equal(bfs.levels(), _oracle(csr, s))
            for k in opt:
                bfs.engine.set_option(k, 1)


@pytest.mark.parametrize("predict", [1, 0])
@pytest.mark.parametrize("mode", ["td", "bu", "do"])
def test_device_loop_matches_host_loop(rt, mode, predict):
    # the device-driven level loop (LevelCtrl decisions on the device) must
    # take exactly the host loop's decisions: same levels, same per-level records
    # (with either direction predictor: mispredictions only cost no-op chains)
    p = dbfs.rmat_params(12, 16, 41)
    csr = dbfs.host_csr_from_params(p)
    dev = dbfs.BFS(p, rt, mode=mode)
    dev.engine.set_option("device_loop_predict", predict)
    host = dbfs.BFS(p, rt, mode=mode)
    host.engine.set_option("device_loop", 0)
    assert dict(dev.engine.get_options())["device_loop"] == 1.0
    for src in dev.sample_roots(4, seed=3) + [0]:
        a, b = dev.run(src), host.run(src)
        assert np.array_equal(dev.levels(), _oracle(csr, src))
        assert np.array_equal(host.levels(), dev.levels())
        strip = lambda r: [(l["dir"], l["frontier"], l["frontier_edges"], l["discovered"]) for l in r.levels]
        assert strip(a) == strip(b)
        assert (a.reached, a.edges, a.depth) == (b.reached, b.edges, b.depth)


def test_host_loop_stats_mailbox():
    # host loop on 3 virtual ranks: level totals read through the mapped
    # mailbox give the oracle's levels; with phase timing
    # every level reports its collective time (comm_ms <= ms)
    p = dbfs.rmat_params(11, 16, 19)
    csr = dbfs.host_csr_from_params(p)
    deg = np.diff(np.asarray(csr.row_off))
    srcs = [int(v) for v in np.nonzero(deg > 0)[0][[0, 50, 400]]]

    def body(rt):
        bfs = dbfs.BFS(p, rt, mode="do")
        bfs.engine.set_option("device_loop", 0)  # the host loop (several ranks default to the device loop)
        bfs.engine.phase_timing = True
        out = []
        for s in srcs:
            res = bfs.run(s)
            out.append((bfs.levels(), res.levels))
        return out

    for rank_out in run_virtual_ranks(3, body, device="cpu"):
        for (lv, levels), s in zip(rank_out, srcs):
            assert np.array_equal(lv, _oracle(csr, s))
            assert levels and all(0.0 <= l["comm_ms"] <= l["ms"] + 1e-6 for l in levels)
            assert any(l["comm_ms"] > 0 for l in levels)


def _mixed_graph(n=20000, seed=7):
    """Hub + long path + random blob: sparse, dense and bottom-up levels in one
    traversal from vertex 0 (degree 3000 > one 2048-edge block)."""
    rng = np.random.default_rng(seed)
    u = [np.zeros(3000, np.int64), np.arange(3000, 6000), rng.integers(6000, n, 40000)]
    v = [np.arange(1, 3001), np.arange(3001, 6001), rng.integers(6000, n, 40000)]
    return n, np.concatenate(u), np.concatenate(v)


@pytest.mark.parametrize("predict", [1, 0])
@pytest.mark.parametrize("mode", ["td", "do"])
@pytest.mark.parametrize("sparse_edges", [0, 1, 64, 4096, 1 << 40])
def test_sparse_top_down_levels(rt, mode, predict, sparse_edges):
    # sparse top-down levels (one kernel: direct claims, work list handed to
    # the next level) mixed with dense and bottom-up levels in any order: the
    # levels and per-level records equal the host loop's
    n, u, v = _mixed_graph()
    g = dbfs.build_csr(n, u, v)
    dev = dbfs.BFS(g, rt, mode=mode)
    dev.engine.set_option("device_loop_predict", predict)
    dev.engine.set_option("td_sparse_edges", sparse_edges)
    host = dbfs.BFS(g, rt, mode=mode)
    host.engine.set_option("device_loop", 0)
    for src in (0, 2999, 4500, 12345):
        a, b = dev.run(src), host.run(src)
        assert np.array_equal(dev.levels(), dbfs.cpu_bfs(g, src)[0])
        strip = lambda r: [(l["dir"], l["frontier"], l["frontier_edges"], l["discovered"]) for l in r.levels]
        assert strip(a) == strip(b)
        assert (a.reached, a.edges, a.depth) == (b.reached, b.edges, b.depth)
    assert dev.validate(12345)


@pytest.mark.parametrize("mode", ["td", "bu", "do"])
def test_narrow_epochs_stale_bytes(rt, mode):
    # level bytes are base + level with a base per run (narrow_epochs): runs
    # alternate between two components (a 62-level path: the deepest narrow
    # traversal, and a 40-level one) so every run meets the other
    # component's and its own earlier epochs' bytes; levels must match the
    # oracle every time (depth 62 fits the bytes: no fallback to wide levels)
    n1, n2 = 63, 41
    src_e = np.concatenate([np.arange(n1 - 1), n1 + np.arange(n2 - 1)])
    dst_e = src_e + 1
    csr = dbfs.build_csr(n1 + n2, src_e, dst_e)
    b = dbfs.BFS(csr, rt, mode=mode)
    for i in range(11):
        src = (0, n1, n1 - 1, n1 + 20)[i % 4]
        r = b.run(src)
        exp = _oracle(csr, src)
        assert np.array_equal(b.levels(), exp), (i, src)
        assert r.depth == int(exp[exp != dbfs.UNREACHED].max()) + 1


@pytest.mark.parametrize("device_loop", [1, 0])
@pytest.mark.parametrize("mode", ["td", "bu", "do"])
def test_narrow_levels(rt, mode, device_loop):
    # one-byte levels during the traversal, widened on read: same levels as
    # the 32-bit array; a path deeper than 62 levels is rerun with 32-bit
    # levels (reported time covers both runs) and later runs stay wide
    p = dbfs.rmat_params(11, 16, 5)
    csr = dbfs.host_csr_from_params(p)
    narrow, wide = dbfs.BFS(p, rt, mode=mode), dbfs.BFS(p, rt, mode=mode)
    wide.engine.set_option("narrow_levels", 0)
    for b in (narrow, wide):
        b.engine.set_option("device_loop", device_loop)
    for src in narrow.sample_roots(9, seed=2):  # > kNarrowEpochs: cycles the byte base
        a, b = narrow.run(src), wide.run(src)
        assert np.array_equal(narrow.local_levels(), wide.local_levels())
        assert np.array_equal(narrow.levels(), _oracle(csr, src))
        assert (a.reached, a.edges, a.depth) == (b.reached, b.edges, b.depth)
        assert narrow.validate(src)
    n = 700
    path = dbfs.build_csr(n, np.arange(n - 1), np.arange(1, n))
    deep = dbfs.BFS(path, rt, mode=mode)
    deep.engine.set_option("device_loop", device_loop)
    for src in (0, 350):
        r = deep.run(src)
        exp = np.abs(np.arange(n) - src)
        assert np.array_equal(deep.levels(), exp)
        assert r.depth == exp.max() + 1 and r.reached == n


@pytest.mark.parametrize("predict", [1, 0])
@pytest.mark.parametrize("mode", ["td", "bu", "do"])
@pytest.mark.parametrize("P", [2, 3])
def test_device_loop_several_ranks(P, mode, predict):
    # the device-driven loop with collectives in every level chain (all-gather,
    # all-to-all, totals all-reduce + level_finish) takes the host loop's
    # decisions on every rank: same levels, records, reached / edges / depth
    p = dbfs.rmat_params(11, 16, 29)
    csr = dbfs.host_csr_from_params(p)
    deg = np.diff(np.asarray(csr.row_off))
    srcs = [int(v) for v in np.nonzero(deg > 0)[0][[0, 77, 901]]]

    def body(rt):
        dev, host = dbfs.BFS(p, rt, mode=mode), dbfs.BFS(p, rt, mode=mode)
        dev.engine.set_option("device_loop_predict", predict)
        dev.engine.set_option("td_byte_edges", 1 << 10)  # byte-map levels (pack + exchange) too
        host.engine.set_option("device_loop", 0)
        out = []
        for s in srcs:
            a, b = dev.run(s), host.run(s)
            strip = lambda r: [(l["dir"], l["frontier"], l["frontier_edges"], l["discovered"]) for l in r.levels]
            out.append((dev.levels(), host.levels(), strip(a), strip(b), (a.reached, a.edges, a.depth),
                        (b.reached, b.edges, b.depth)))
        return out

    for rank_out in run_virtual_ranks(P, body, device="cpu"):
        for (ld, lh, ra, rb, ta, tb), s in zip(rank_out, srcs):
            assert np.array_equal(ld, _oracle(csr, s)) and np.array_equal(lh, ld)
            # (the device loop stops once every vertex with an edge is reached:
            # the host loop's extra last level expanded its frontier for nothing)
            assert ra == rb[:len(ra)] and all(r[3] == 0 for r in rb[len(ra):]) and ta == tb


@pytest.mark.parametrize("knobs", [
    {},                                             # defaults: sparse list levels, gathered bottom-up inputs
    {"list_form_edges": 0},                         # dense top-down chains only
    {"list_form_edges": 64},                        # lists too small: sparse chains re-enqueued dense
    {"xsparse_edges": 0},                           # only level 0 predicted sparse
    {"device_loop_predict": 0},                     # no prediction: two wasted chains per switch
])
@pytest.mark.parametrize("P", [2, 3, 8])
def test_device_loop_sparse_lists_several_ranks(P, knobs):
    """Several ranks, device loop: sparse top-down levels (owned targets
    settled in place, remote ones appended to owner lists exchanged
    count-sized, settled on their owners by td_sparse_apply; the lists'
    capacity checked against the global frontier edges on every rank), the
    frontier all-gathered by the collective of the level before a bottom-up
    one, and fused finishes -- the host loop's levels and records."""
    p = dbfs.rmat_params(12, 16, 31)
    csr = dbfs.host_csr_from_params(p)
    deg = np.diff(np.asarray(csr.row_off))
    srcs = [int(v) for v in np.nonzero(deg > 0)[0][[0, 55, 700, 1500]]]

    def body(rt):
        dev, host = dbfs.BFS(p, rt, mode="do"), dbfs.BFS(p, rt, mode="do")
        for k, v in knobs.items():
            dev.engine.set_option(k, v)
        host.engine.set_option("device_loop", 0)
        assert dev.graph.nhubs > 0
        out = []
        for s in srcs:
            a, b = dev.run(s), host.run(s)
            strip = lambda r: [(l["dir"], l["frontier"], l["frontier_edges"], l["discovered"]) for l in r.levels]
            out.append((dev.levels(), strip(a), strip(b), (a.reached, a.edges, a.depth), (b.reached, b.edges, b.depth),
                        a.mispredicts, [c[1] for c in a.chains]))
        return out

    for rank_out in run_virtual_ranks(P, body, device="cpu"):
        mis = 0
        forms = ""
        for (ld, ra, rb, ta, tb, m, fs), s in zip(rank_out, srcs):
            assert np.array_equal(ld, _oracle(csr, s))
            # (the device loop stops once every vertex with an edge is reached)
            assert ra == rb[:len(ra)] and all(r[3] == 0 for r in rb[len(ra):]) and ta == tb
            mis += m
            forms += "".join(fs)
        if knobs.get("list_form_edges", 1) == 64:
            assert mis > 0  # undersized sparse chains were replaced
        if knobs.get("list_form_edges", 1) == 0:
            assert "S" not in forms
        elif knobs.get("device_loop_predict", 1):
            assert "S" in forms


@pytest.mark.parametrize("P", [2, 3])
def test_bottom_up_mode_split_several_ranks(P):
    """bu mode on several ranks: the seed's reduction carries the hub bits, so
    level 0 is already a split bottom-up level."""
    p = dbfs.rmat_params(11, 16, 13)
    csr = dbfs.host_csr_from_params(p)
    deg = np.diff(np.asarray(csr.row_off))
    srcs = [int(v) for v in np.nonzero(deg > 0)[0][[3, 400]]]

    def body(rt):
        b = dbfs.BFS(p, rt, mode="bu")
        return [(b.run(s), b.levels())[1] for s in srcs]

    for rank_out in run_virtual_ranks(P, body, device="cpu"):
        for lv, s in zip(rank_out, srcs):
            assert np.array_equal(lv, _oracle(csr, s))


@pytest.mark.parametrize("case", [(1, [], [], 0), (2, [0], [1], 1), (5, [0, 1], [1, 2], 4),
                                  (130, list(range(128)), list(range(1, 129)), 129),
                                  (130, list(range(128)), list(range(1, 129)), 0)])
def test_tiny_and_isolated_sources(rt, case):
    # one-vertex graph, isolated sources, a slice boundary inside a path: every
    # mode (device loop: sparse levels, narrow levels) on one rank and three
    n, u, v, src = case
    g = dbfs.build_csr(n, np.array(u, dtype=np.int64), np.array(v, dtype=np.int64))
    exp = dbfs.cpu_bfs(g, src)[0]
    for mode in ("td", "bu", "do"):
        b = dbfs.BFS(g, rt, mode=mode)
        b.run(src)
        assert np.array_equal(b.levels(), exp)

    def body(r):
        b = dbfs.BFS(g, r, mode="do")
        b.run(src)
        return b.levels()

    for lv in run_virtual_ranks(3, body, device="cpu"):
        assert np.array_equal(lv, exp)


@pytest.mark.parametrize("mode", ["td", "do"])
@pytest.mark.parametrize("direct_edges", [0, 1 << 40])
def test_td_direct_levels_cpu(rt, mode, direct_edges):
    p = dbfs.rmat_params(12, 16, 38)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, rt, mode=mode)
    bfs.engine.set_option("td_direct_edges", direct_edges)
    for s in (0, 9, 3000):
        bfs.run(s)
        assert np.array_equal(bfs.levels(), _oracle(csr, s))
    n = 400
    chain = dbfs.build_csr(n, np.arange(n - 1, dtype=np.uint32), np.arange(1, n, dtype=np.uint32))
    cb = dbfs.BFS(chain, rt, mode=mode)
    cb.engine.set_option("td_direct_edges", direct_edges)
    cb.run(0)
    assert np.array_equal(cb.levels(), np.arange(n))


@pytest.mark.parametrize("mode", ["do", "td"])
def test_td_fused_finish_cpu(rt, mode):
    # dense top-down levels finished in the update (unit prefixes deferred to
    # the next compaction): exact
    p = dbfs.rmat_params(12, 16, 67)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, rt, mode=mode)
    for src in bfs.sample_roots(3, seed=9):
        bfs.run(src)
        assert np.array_equal(bfs.levels(), dbfs.cpu_bfs(csr, src)[0])


def test_validator_counts(rt):
    # Graph500 validator: clean levels -> no violations; validated against
    # another source, exactly the two vertices with the wrong level-0 status
    p = dbfs.rmat_params(11, 16, 9)
    b = dbfs.BFS(p, rt, mode="do")
    src, other = b.sample_roots(2, seed=8)
    b.run(src)
    assert list(b.engine.validate(int(src))) == [0, 0, 0]
    assert list(b.engine.validate(int(other))) == [0, 0, 2]


def test_run_many_matches_single_runs(rt):
    """run_many: back-to-back traversals in native code give the same per-run
    results as one run() per source, and the last one's levels stay readable."""
    p = dbfs.rmat_params(11, 16, 13)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, rt, mode="do")
    srcs = bfs.sample_roots(5, seed=3)
    singles = [bfs.run(s) for s in srcs]
    many = bfs.run_many(srcs)
    assert [r.source for r in many] == list(srcs)
    for a, b in zip(singles, many):
        assert (a.reached, a.edges, a.depth) == (b.reached, b.edges, b.depth)
    assert np.array_equal(bfs.levels(), _oracle(csr, srcs[-1]))


@pytest.mark.parametrize("bits", [1, 0])
@pytest.mark.parametrize("P", [1, 3])
def test_sparse_level_from_bitmap(P, bits):
    """A sparse top-down level right after a bottom-up one reads the bottom-up
    output bitmap itself (td_sparse_bits: no unit scan / compaction) or a
    compacted work list (0): same levels and per-level records, exact against
    the oracle, with one and several ranks; such a level occurs."""
    p = dbfs.rmat_params(12, 16, 31)
    csr = dbfs.host_csr_from_params(p)
    deg = np.diff(np.asarray(csr.row_off))
    srcs = [int(v) for v in np.nonzero(deg > 0)[0][[3, 500, 1700]]]

    def body(rt):
        b = dbfs.BFS(p, rt, mode="do")
        b.engine.set_option("td_sparse_bits", bits)
        out = []
        for s in srcs:
            r = b.run(s)
            forms = "".join(c[1] for c in r.chains)
            out.append((b.levels(), [(l["dir"], l["frontier"], l["frontier_edges"]) for l in r.levels], forms))
        return out

    ref = None
    if P == 1:
        results = [body(init_runtime("cpu"))]
    else:
        results = run_virtual_ranks(P, body, device="cpu")
    for rank_out in results:
        for (lv, recs, forms), s in zip(rank_out, srcs):
            assert np.array_equal(lv, _oracle(csr, s))
        assert any("BS" in forms for _, _, forms in rank_out)
        ref = ref or [recs for _, recs, _ in rank_out]
        assert [recs for _, recs, _ in rank_out] == ref


@pytest.mark.parametrize("narrow", [1, 0])
@pytest.mark.parametrize("max_hubs", [300, None])
@pytest.mark.parametrize("cut_edges", [0, 1 << 40])
@pytest.mark.parametrize("alpha", [24.0, 1e9, 2.0])
def test_hub_cut_bottom_up_levels(rt, cut_edges, alpha, max_hubs, narrow):
    """Hub-cut bottom-up levels (BuArgs::cut_edges): the non-hub frontier's
    neighbours claimed top-down, rows resolved by frontier hubs only, the two
    merged -- levels, reached vertices and edges exact, with the cut taken on
    every first bottom-up level (1 << 40) or never (0); alpha moves the switch
    from the first levels (1e9: bottom-up right after the root) to late ones;
    300 hubs leave most frontier vertices to the top-down part, the default
    cap makes every vertex with an edge a hub; narrow levels keep the claims
    in the level bytes, wide ones in a claim-byte array."""
    p = dbfs.rmat_params(13, 16, 11)
    csr = dbfs.host_csr_from_params(p)
    deg = np.diff(np.asarray(csr.row_off))
    bfs = dbfs.BFS(p, rt, mode="do", alpha=alpha, beta=24.0, max_hubs=max_hubs)
    bfs.engine.set_option("bu_cut_edges", cut_edges)
    bfs.engine.set_option("narrow_levels", narrow)
    assert bfs.graph.nhubs > 0
    for src in bfs.sample_roots(6, seed=3):
        res = bfs.run(src)
        exp = _oracle(csr, src)
        assert np.array_equal(bfs.levels(), exp)
        assert res.reached == int((exp != dbfs.UNREACHED).sum())
        assert res.edges == int(deg[exp != dbfs.UNREACHED].sum()) // 2
        assert "B" in "".join(l["dir"] for l in res.levels)
        assert bfs.validate(src)


@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("narrow", [1, 0])
def test_hub_cut_several_ranks(P, narrow):
    """The hub cut with several ranks (EngineOptions::bu_cut_ranks): every
    rank claims its own non-hub frontier's neighbours, the remote ones packed
    per owner and all-to-all'ed, merged on the owners (bu_cut_merge) -- forced
    on every first bottom-up level (bu_cut_edges 2^40, any prediction), then
    off (bu_cut_ranks 1): levels exact against the oracle both ways, the level
    records equal, and the cut chains enqueued only when allowed.  300 hubs
    leave most frontier vertices to the top-down part; narrow levels keep the
    claims in the level bytes, wide ones in the claim bytes."""
    p = dbfs.rmat_params(13, 16, 11)
    csr = dbfs.host_csr_from_params(p)
    srcs = [7, 3001, 8100]

    def body(rt):
        b = dbfs.BFS(p, rt, mode="do", alpha=2.0, beta=24.0, max_hubs=300)
        b.engine.set_option("narrow_levels", narrow)
        b.engine.set_option("bu_cut_edges", 1 << 40)
        b.engine.set_option("bu_cut_mf_frac", 1.0)
        out = []
        for ranks in (8, 1):  # (8: at least P)
            b.engine.set_option("bu_cut_ranks", ranks)
            for s in srcs:
                r = b.run(s)
                recs = [(l["dir"], l["frontier"], l["frontier_edges"], l["discovered"]) for l in r.levels]
                out.append((ranks, s, b.levels(), recs, sum(1 for c in r.chains if c[7])))
        return out

    for outs in run_virtual_ranks(P, body, device="cpu"):
        cut = {s: x for c, s, *x in outs if c == 8}
        plain = {s: x for c, s, *x in outs if c == 1}
        for s in srcs:
            exp = dbfs.cpu_bfs(csr, s)[0]
            assert np.array_equal(cut[s][0], exp) and np.array_equal(plain[s][0], exp)
            assert cut[s][1] == plain[s][1]
            assert plain[s][2] == 0
        assert sum(cut[s][2] for s in srcs) > 0


@pytest.mark.parametrize("n,m,mode", [(3000, 30000, "td"), (600011, 2400000, "td"), (600011, 2400000, "do")])
def test_unvisited_filter_levels_cpu(n, m, mode):
    """The unvisited filter (UnvisArgs, TdArgs::unvis) on the CPU backend:
    forced on every dense top-down level (td_unvis_edges 1, any visited
    fraction), the CPU expansion skips a target whose filter bit is clear --
    so a filter bit lost for an unvisited vertex shows as a wrong level.
    Identity mapping (n <= kUnvisBits) and the multiply-shift runs (n >
    kUnvisBits, an n that is no power of two); one rank and 3 virtual ranks."""
    from distributed_cuda_bfs_amd.parallel.runtime import run_virtual_ranks

    p = dbfs.uniform_params(n, m, 17)
    csr = dbfs.host_csr_from_params(p)
    roots = [1, n // 3, n - 5]
    exp = {s: dbfs.cpu_bfs(csr, s)[0] for s in roots}

    def body(rt):
        b = dbfs.BFS(p, rt, mode=mode)
        b.engine.set_option("td_unvis_edges", 1)
        b.engine.set_option("td_unvis_vis_frac", 0.0)
        b.engine.set_option("td_unvis_max_density", 1.0)
        b.engine.set_option("td_sparse_edges", 0)
        used = False
        for s in roots:
            r = b.run(s)
            assert np.array_equal(b.levels(), exp[s]), (rt.rank, s)
            used = used or any(c[5] for c in r.chains)
        return used

    for P in (1, 3):
        assert all(run_virtual_ranks(P, body, device="cpu"))


@pytest.mark.parametrize("P", [1, 3])
def test_power_law_generator(P):
    """Chung-Lu power-law graphs (power_law_params): labels scrambled into
    [0, n) for an n that is no power of two, a heavy-tailed degree sequence
    whose top expected degree follows dmax, and levels exact against the oracle
    on one rank and on virtual ranks (the shard build regenerates the same
    edges as the host copy)."""
    p = dbfs.power_law_params(30011, 420000, 1500, 5)
    assert p.power_law and p.pl_i0 > 0
    csr = dbfs.host_csr_from_params(p)
    deg = np.diff(np.asarray(csr.row_off))
    assert deg.sum() == 2 * 420000
    assert 0.5 * 1500 < deg.max() < 2.0 * 1500 and deg.max() > 20 * deg.mean()
    u, v = dbfs.generate_edges(p, 0, 1000)
    assert np.asarray(u).max() < 30011 and np.asarray(v).max() < 30011
    srcs = [int(np.argmax(deg)), 4]

    def body(rt):
        b = dbfs.BFS(p, rt, mode="do")
        return [(b.run(s), b.levels())[1] for s in srcs]

    outs = [body(dbfs.init_runtime("cpu"))] if P == 1 else run_virtual_ranks(P, body, device="cpu")
    for rank_out in outs:
        for lv, s in zip(rank_out, srcs):
            assert np.array_equal(lv, _oracle(csr, s))


@pytest.mark.parametrize("parts", [2, 3])
@pytest.mark.parametrize("mode", ["td", "do"])
def test_split_levels_cpu(parts, mode):
    """Split top-down levels (TdArgs::split_k, refresh_visited) on the CPU
    backend: every level-byte top-down level of at least one frontier edge
    forced into `parts` parts (2 x parts past 16 x the threshold), the
    claims so far ORed into visited between them and the update taking every level byte as new -- levels exact against
    the oracle, and the chain records show the split."""
    p = dbfs.rmat_params(14, 16, 23)
    csr = dbfs.host_csr_from_params(p)
    roots = [0, 77, 9000]
    b = dbfs.BFS(p, init_runtime("cpu"), mode=mode)
    b.engine.set_heuristics(24.0, 24.0, 8, td_byte_edges=0)
    b.engine.set_option("td_split_edges", 1)
    b.engine.set_option("td_split_parts", parts)
    b.engine.set_option("td_sparse_edges", 0)
    used = False
    for s in roots:
        r = b.run(s)
        assert np.array_equal(b.levels(), dbfs.cpu_bfs(csr, s)[0]), s
        used = used or any(c[6] in (parts, 2 * parts) for c in r.chains)
    assert used


def test_grid_generator_shape():
    # 2-D grid (road-like): row-major labels, right and lower neighbours
    p = dbfs.grid_params(7, 5)
    assert p.n == 35 and p.m == 6 * 5 + 7 * 4
    csr = dbfs.host_csr_from_params(p)
    deg = np.diff(np.asarray(csr.row_off)).reshape(5, 7)
    assert deg[0, 0] == 2 and deg[2, 3] == 4 and deg[0, 3] == 3
    lv = _oracle(csr, 0).reshape(5, 7)
    assert np.array_equal(lv, np.add.outer(np.arange(5), np.arange(7)))


@pytest.mark.parametrize("mode", ["td", "do", "bu"])
@pytest.mark.parametrize("P", [1, 3])
def test_high_diameter_grid(mode, P):
    """A 48 x 40 grid: 86 levels from a corner (past the one-byte levels'
    62: the traversal reruns with 32-bit levels), tiny frontiers throughout
    -- the per-level path every level takes; exact against the oracle, on one
    and on three virtual ranks."""
    p = dbfs.grid_params(48, 40)
    csr = dbfs.host_csr_from_params(p)
    srcs = [0, 48 * 20 + 24, 48 * 40 - 1]
    exp = [_oracle(csr, s) for s in srcs]

    def body(rt):
        bfs = dbfs.BFS(p, rt, mode=mode)
        out = []
        for s in srcs:
            r = bfs.run(s)
            out.append((bfs.levels(), r.depth))
        return out

    for rank_out in run_virtual_ranks(P, body, device="cpu"):
        for (lv, depth), e in zip(rank_out, exp):
            assert np.array_equal(lv, e)
            assert depth == int(e.max()) + 1
