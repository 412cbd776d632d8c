"""GPU correctness of the hand-written gfx950 kernels through the engine.

Every test compares the GPU levels against the sequential CPU oracle (the
reference's bfsCPU, bfs.cu:923-945) element-wise -- the reference's own
checkOutput contract (bfs.cu:374-384).
"""
import os

import numpy as np
import pytest

import distributed_cuda_bfs_amd as dbfs
from distributed_cuda_bfs_amd.parallel.runtime import init_runtime, run_virtual_ranks

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

MODES = ["do", "td", "bu", "ref", "simple", "scan"]


def _describe(src, res, got, exp):
    """A levels mismatch, self-described: the root, the first mismatching
    vertices, the chains the device loop enqueued and its level records."""
    bad = np.nonzero(got != exp)[0]
    first = ", ".join(f"{int(v)}: {int(got[v])} vs {int(exp[v])}" for v in bad[:8])
    recs = []
    if res is not None:
        for r in res.levels:
            recs.append(f"[{r.get('level')} {r.get('dir')} nf={r.get('frontier')} mf={r.get('frontier_edges')} "
                        f"new={r.get('discovered')}]")
    chains = [f"{c[0]}{c[1]}:{c[2]}" for c in res.chains] if res is not None else []
    return (f"root {src}: {bad.size} vertices differ (got vs expected: {first}); "
            f"chains {' '.join(chains)}; records {' '.join(recs)}")


def _check(bfs, csr, src):
    res = bfs.run(src)
    exp, _ = dbfs.cpu_bfs(csr, src)
    got = bfs.levels()
    assert np.array_equal(got, exp), _describe(src, res, got, exp)
    reached = int(np.count_nonzero(exp != dbfs.UNREACHED))
    assert res.reached == reached
    ro = np.asarray(csr.row_off)
    deg = np.diff(ro)
    assert res.edges == int(deg[exp != dbfs.UNREACHED].sum()) // 2
    return res


def test_native_is_hip(gpu_runtime):
    assert gpu_runtime.backend.is_gpu
    assert "gfx950" in gpu_runtime.backend.name


@pytest.mark.parametrize("mode", MODES)
def test_chain8(gpu_runtime, data_dir, mode):
    csr = dbfs.read_graph(f"{data_dir}/chain8.txt")
    bfs = dbfs.BFS(csr, gpu_runtime, mode=mode)
    res = _check(bfs, csr, 0)
    assert res.depth == 8
    assert list(bfs.levels()) == list(range(8))


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("scale,seed", [(10, 1), (14, 2), (17, 3)])
def test_rmat_modes(gpu_runtime, mode, scale, seed):
    p = dbfs.rmat_params(scale, 16, seed)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, gpu_runtime, mode=mode)
    for src in bfs.sample_roots(3, seed=seed):
        _check(bfs, csr, src)
    assert bfs.validate(src)


@pytest.mark.parametrize("mode", ["do", "td", "bu"])
def test_uniform_and_isolated_source(gpu_runtime, mode):
    p = dbfs.uniform_params(5000, 12000, 9)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, gpu_runtime, mode=mode)
    deg = np.diff(np.asarray(csr.row_off))
    iso = np.nonzero(deg == 0)[0]
    srcs = [int(np.argmax(deg)), 0] + ([int(iso[0])] if iso.size else [])
    for s in srcs:
        _check(bfs, csr, s)


@pytest.mark.parametrize("mode", ["td", "do"])
def test_all_reached_stop(gpu_runtime, mode):
    """A connected graph (every vertex has an edge, one component): the device
    loop stops once every vertex with an edge is reached instead of expanding
    the last frontier; levels, reached vertices, edges and depth stay exact
    -- a uniform graph of mean degree 28 (the LiveJournal-sized shape, scaled
    down) and a power-law one, 32-bit levels too."""
    for p in (dbfs.uniform_params(300000, 4200000, 5), dbfs.power_law_params(300007, 4200000, 4000, 9)):
        csr = dbfs.host_csr_from_params(p)
        deg = np.diff(np.asarray(csr.row_off))
        bfs = dbfs.BFS(p, gpu_runtime, mode=mode)
        for narrow in (1, 0):
            bfs.engine.set_option("narrow_levels", narrow)
            for s in (int(np.argmax(deg)), 12345, 299000):
                res = _check(bfs, csr, s)
                exp, _ = dbfs.cpu_bfs(csr, s)
                assert res.depth == int(exp[exp != dbfs.UNREACHED].max()) + 1
                assert bfs.validate(s)


@pytest.mark.parametrize("forced", [False, True])
def test_unvisited_filter_gpu(gpu_runtime, forced):
    """Dense top-down levels with the LDS unvisited filter (unvis_filter_kernel
    + td_expand's kUnvis variant): exact levels, reached vertices and edges on
    a uniform graph larger than the filter (multiply-shift runs), a power-law
    one and RMAT-18 (32-bit levels too); by default on the late large levels
    (a uniform graph of mean degree 28 has one), forced: every dense level."""
    graphs = [dbfs.uniform_params(1500007, 21000000, 5), dbfs.power_law_params(600011, 8400000, 6000, 9),
              dbfs.rmat_params(18, 16, 3)]
    used = False
    for p in graphs:
        csr = dbfs.host_csr_from_params(p)
        deg = np.diff(np.asarray(csr.row_off))
        bfs = dbfs.BFS(p, gpu_runtime, mode="td")
        if forced:
            bfs.engine.set_option("td_unvis_edges", 1)
            bfs.engine.set_option("td_unvis_vis_frac", 0.0)
            bfs.engine.set_option("td_unvis_max_density", 1.0)
        for narrow in (1, 0):
            bfs.engine.set_option("narrow_levels", narrow)
            for s in (int(np.argmax(deg)), 12345):
                res = _check(bfs, csr, s)
                used = used or any(c[5] for c in res.chains)
                assert bfs.validate(s)
    assert used


def test_hub_heavy_star(gpu_runtime):
    # one vertex with degree >> kTdEdgesPerBlock exercises multi-block hubs
    n = 50000
    u = np.zeros(n - 1, dtype=np.uint32)
    v = np.arange(1, n, dtype=np.uint32)
    csr = dbfs.build_csr(n, u, v)
    for mode in ["td", "do", "ref"]:
        bfs = dbfs.BFS(csr, gpu_runtime, mode=mode)
        _check(bfs, csr, 0)
        _check(bfs, csr, 7)


def test_device_generator_matches_host(gpu_runtime):
    p = dbfs.rmat_params(12, 16, 5)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, gpu_runtime)
    dev = bfs.graph.to_host()
    assert np.array_equal(np.asarray(dev.row_off), np.asarray(csr.row_off))
    ro = np.asarray(csr.row_off)
    dc, hc = np.asarray(dev.col), np.asarray(csr.col)
    for r in range(0, csr.n, 97):  # same multiset per row (device fill order is atomic-ordered)
        assert np.array_equal(np.sort(dc[ro[r]:ro[r + 1]]), np.sort(hc[ro[r]:ro[r + 1]]))


def test_power_law_generator_on_device(gpu_runtime):
    """The Chung-Lu power-law generator (the soc-LiveJournal1 / Friendster
    stand-in, integer-only inverse CDF): the device-built shard equals the host
    copy row for row, and every mode's levels equal the oracle from the
    hubs, a low-degree vertex and 3 virtual ranks."""
    p = dbfs.power_law_params(200003, 2900000, 6000, 3)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, gpu_runtime)
    dev = bfs.graph.to_host()
    assert np.array_equal(np.asarray(dev.row_off), np.asarray(csr.row_off))
    deg = np.diff(np.asarray(csr.row_off))
    assert deg.max() > 20 * deg.mean()  # (a heavy tail, not a uniform graph)
    for mode in ("do", "td", "bu"):
        bfs.mode = mode
        for s in (int(np.argmax(deg)), int(np.argmin(np.where(deg > 0, deg, 1 << 30)))):
            _check(bfs, csr, s)
    srcs = [int(np.argmax(deg)), 17]

    def body(rt):
        b = dbfs.BFS(p, rt, mode="do")
        return [(b.run(s), b.levels())[1] for s in srcs]

    for rank_out in run_virtual_ranks(3, body, device="hip"):
        for lv, s in zip(rank_out, srcs):
            assert np.array_equal(lv, dbfs.cpu_bfs(csr, s)[0])


@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("mode", ["do", "td", "ref"])
def test_virtual_ranks_on_one_gpu(P, mode):
    p = dbfs.rmat_params(13, 16, 11)
    csr = dbfs.host_csr_from_params(p)
    src = 5
    exp, _ = dbfs.cpu_bfs(csr, src)

    def body(rt):
        bfs = dbfs.BFS(p, rt, mode=mode)
        bfs.run(src)
        return bfs.levels()

    outs = run_virtual_ranks(P, body, device="hip")
    for o in outs:
        assert np.array_equal(o, exp)


@pytest.mark.parametrize("mode", ["do", "ref"])
def test_parent_tree_gpu(gpu_runtime, mode):
    from distributed_cuda_bfs_amd.utils.validate import parents_are_valid

    p = dbfs.rmat_params(12, 16, 21)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, gpu_runtime, mode=mode)
    src = bfs.sample_roots(1, seed=8)[0]
    bfs.run(src)
    assert parents_are_valid(csr, bfs.levels(), bfs.parents(src), src)


def test_cli_gpu_reference_stdout(data_dir):
    import os
    import subprocess

    repo = os.path.dirname(os.path.dirname(data_dir))  # data_dir = <repo>/tests/data
    out = subprocess.run([os.path.join(repo, "bin", "bfs"), "0", os.path.join(data_dir, "chain8.txt")],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "Enabling peer access between GPU0 and GPU1..." in out.stdout
    assert out.stdout.endswith("Output OK!\n\n")


@pytest.mark.parametrize("mode", MODES)
def test_rccl_single_rank_exchange_path(gpu_runtime, mode):
    """RCCL communicator (1 rank) driving the full exchange path: ncclAllToAll,
    in-place ncclAllGather, ncclAllReduce, grouped ncclSend/ncclRecv."""
    from distributed_cuda_bfs_amd.parallel.runtime import Runtime

    N = dbfs.native
    be = gpu_runtime.backend
    comm = N.nccl_comm(N.nccl_unique_id(), 0, 1, be)
    assert comm.name == "rccl"
    rt = Runtime(backend=be, comm=comm)
    p = dbfs.rmat_params(14, 16, 23)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, rt, mode=mode, force_exchange=True)
    for src in bfs.sample_roots(2, seed=6):
        _check(bfs, csr, src)
    assert comm.sum_host(41) == 41 and comm.max_host(2.5) == 2.5
    comm.barrier()


def test_rccl_and_virtual_comm_patterns_gpu(gpu_runtime):
    """Communicator unit exercise (tests/test_comm.py) on device memory: RCCL
    (1 rank) and VirtualComm ranks on one GPU."""
    from test_comm import _check, _exercise

    N = dbfs.native
    be = gpu_runtime.backend
    comm = N.nccl_comm(N.nccl_unique_id(), 0, 1, be)
    _check(_exercise(comm, be, 1, 0), 1, 0)
    outs = run_virtual_ranks(3, lambda rt: _exercise(rt.comm, rt.backend, 3, rt.rank), device="hip")
    for me, res in enumerate(outs):
        _check(res, 3, me)


@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("mode", ["td", "do"])
@pytest.mark.parametrize("knobs", [{}, {"td_check_visited_min": 2.0, "td_wide_below_blocks": 1 << 30},
                                   {"td_check_visited_min": 0.0, "td_wide_below_blocks": 0}])
def test_td_byte_map_mode_gpu(P, mode, knobs):
    # byte map on every top-down level; with / without the visited pre-check,
    # 256- and 1024-thread workgroups
    p = dbfs.rmat_params(16, 16, 29)
    csr = dbfs.host_csr_from_params(p)
    srcs = [0, 5, 40000]
    exp = [dbfs.cpu_bfs(csr, s)[0] for s in srcs]

    def body(rt):
        bfs = dbfs.BFS(p, rt, mode=mode)
        bfs.engine.set_heuristics(24.0, 24.0, 8, td_byte_edges=0)
        for k, v in knobs.items():
            bfs.engine.set_option(k, v)
        out = []
        for s in srcs:
            res = bfs.run(s)
            out.append((s, res, bfs.levels()))
        return out

    for rank_out in run_virtual_ranks(P, body, device="hip"):
        for (s, res, lv), e in zip(rank_out, exp):
            assert np.array_equal(lv, e), _describe(s, res, lv, e)


@pytest.mark.parametrize("mode", ["td", "do"])
def test_sparse_level_late_workgroups_gpu(mode, monkeypatch):
    """Regression for round 5's intermittent wrong levels / missing stamp
    (test_td_byte_map_mode_gpu[*-td-1], root 0 of RMAT-16).  A one-rank
    td_sparse launch finishes its level in its last workgroup; workgroups past
    the level's active count return before the ticket, so one dispatched after
    that finish must not see the next level's totals.  DBFS_FAULT_INJECT
    kind=late_wg makes every such workgroup start 300 us late, which turns the
    rare dispatch order into the only one: with the level's input and output
    totals in one stats block, root 0 (the RMAT hub: a level-0 list of a few
    blocks, a level-1 list of ~250) ran level-1 totals against level 0's
    lists -- vertices one level early and late, and a shifted ticket that left
    a later one-block sparse level without its stamp."""
    monkeypatch.setenv("DBFS_FAULT_INJECT", "kind=late_wg,us=300")
    p = dbfs.rmat_params(16, 16, 29)
    csr = dbfs.host_csr_from_params(p)
    srcs = [0, 5, 40000, 0]
    exp = {s: dbfs.cpu_bfs(csr, s)[0] for s in set(srcs)}

    def body(rt):
        bfs = dbfs.BFS(p, rt, mode=mode)
        bfs.engine.set_heuristics(24.0, 24.0, 8, td_byte_edges=0)
        bfs.engine.set_option("td_check_visited_min", 0.0)
        out = []
        for s in srcs:
            res = bfs.run(s)
            out.append((s, res, bfs.levels()))
        return out

    (rank_out,) = run_virtual_ranks(1, body, device="hip")
    sparse = 0
    for s, res, lv in rank_out:
        assert np.array_equal(lv, exp[s]), _describe(s, res, lv, exp[s])
        sparse += sum(1 for c in res.chains if c[1] == "S")
    assert sparse > 0  # (the injected kernel ran)


@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("mode", ["td", "do"])
def test_sparse_list_exchange_gpu(gpu_runtime, P, mode):
    """Owner-list exchange for every top-down level (P=1 through a 1-rank RCCL
    communicator with force_exchange, P=3 through virtual ranks on one GPU)."""
    from distributed_cuda_bfs_amd.parallel.runtime import Runtime

    p = dbfs.rmat_params(16, 16, 31)
    csr = dbfs.host_csr_from_params(p)
    srcs = [1, 7, 50000]
    exp = [dbfs.cpu_bfs(csr, s)[0] for s in srcs]

    def body(rt):
        bfs = dbfs.BFS(p, rt, mode=mode, force_exchange=True)
        bfs.engine.set_heuristics(24.0, 24.0, 8, sparse_max_edges=1 << 40, sparse_size_check=0)
        out = []
        for s in srcs:
            bfs.run(s)
            out.append(bfs.levels())
        return out

    if P == 1:
        N = dbfs.native
        be = gpu_runtime.backend
        outs = [body(Runtime(backend=be, comm=N.nccl_comm(N.nccl_unique_id(), 0, 1, be)))]
    else:
        outs = run_virtual_ranks(P, body, device="hip")
    for rank_out in outs:
        for lv, e in zip(rank_out, exp):
            assert np.array_equal(lv, e)


def test_hub_sort_gpu_matches_cpu(gpu_runtime):
    from distributed_cuda_bfs_amd.parallel.runtime import init_runtime

    p = dbfs.rmat_params(15, 16, 12)
    gpu = dbfs.BFS(p, gpu_runtime, hub_sort=True)
    cpu = dbfs.BFS(p, init_runtime("cpu"), hub_sort=True)
    g, c = gpu.graph.to_host(), cpu.graph.to_host()
    assert np.array_equal(np.asarray(g.row_off), np.asarray(c.row_off))
    ro = np.asarray(g.row_off)
    gc, cc = np.asarray(g.col), np.asarray(c.col)
    for r in range(g.rows):
        n = ro[r + 1] - ro[r]
        if 2 <= n <= 4096:
            assert np.array_equal(gc[ro[r]:ro[r + 1]], cc[ro[r]:ro[r + 1]]), r


@pytest.mark.parametrize("mode", ["td", "bu", "do"])
@pytest.mark.parametrize("byte_edges", [-1, 0])
def test_device_loop_matches_host_loop_gpu(gpu_runtime, mode, byte_edges):
    """Device-driven level loop (predicated kernels + LevelCtrl decisions in
    the scan's last workgroup + mailbox stamps) against the host loop."""
    p = dbfs.rmat_params(16, 16, 43)
    csr = dbfs.host_csr_from_params(p)
    dev = dbfs.BFS(p, gpu_runtime, mode=mode)
    host = dbfs.BFS(p, gpu_runtime, mode=mode)
    host.engine.set_option("device_loop", 0)
    for b in (dev, host):
        b.engine.set_heuristics(24.0, 24.0, 8, td_byte_edges=byte_edges)
        b.engine.phase_timing = True
    for src in dev.sample_roots(4, seed=5):
        a = dev.run(src)
        exp = dbfs.cpu_bfs(csr, src)[0]
        assert np.array_equal(dev.levels(), exp)
        r = host.run(src)
        strip = lambda x: [(l["dir"], l["frontier"], l["frontier_edges"], l["discovered"]) for l in x.levels]
        assert strip(a) == strip(r)
        assert (a.reached, a.edges, a.depth) == (r.reached, r.edges, r.depth)
        assert all(l["ms"] > 0 for l in a.levels)


@pytest.mark.parametrize("lane_limit", [1, 8, 64])
def test_bottom_up_variants_gpu(gpu_runtime, lane_limit):
    """Bottom-up phase 2 (the wave scans unresolved rows one at a time) after
    per-lane phases of several lengths, pure BU and direction-optimising."""
    p = dbfs.rmat_params(17, 16, 47)
    csr = dbfs.host_csr_from_params(p)
    for mode in ["bu", "do"]:
        bfs = dbfs.BFS(p, gpu_runtime, mode=mode, bu_lane_limit=lane_limit)
        for src in bfs.sample_roots(3, seed=lane_limit):
            _check(bfs, csr, src)


def test_perf_regression_do_vs_ref_gpu(gpu_runtime):
    """SURVEY §7.4 perf guard: on RMAT-18 the direction-optimising engine must
    stay far ahead of the reference algorithm on the same GPU (measured
    ~100x at RMAT-26; require 10x here to stay robust on a shared box)."""
    p = dbfs.rmat_params(18, 16, 3)
    ref = dbfs.BFS(p, gpu_runtime, mode="ref")
    do = dbfs.BFS(p, gpu_runtime, mode="do")
    roots = do.sample_roots(4, seed=2)
    for b in (ref, do):
        b.run(roots[0])  # warm-up
    t_ref = sum(ref.run(r).ms for r in roots)
    t_do = sum(do.run(r).ms for r in roots)
    assert t_do * 10 < t_ref, (t_do, t_ref)


@pytest.mark.parametrize("whole,small", [(1, 0), (-1, -1), (-1, 1)])
@pytest.mark.parametrize("max_hubs", [None, 64, 3000, 0])
def test_bottom_up_hub_lds_gpu(gpu_runtime, max_hubs, whole, small):
    """Bottom-up with hub-encoded heads probed in the LDS copy of the hub
    frontier bits: every vertex a hub (default cap on a small graph), a few
    hubs (mixed LDS / global head probes), no hubs (plain kernel); whole
    64-word units per wave, or units split at 16 / 4 words per wave
    (bu_small_waves)."""
    p = dbfs.rmat_params(16, 16, 53)
    csr = dbfs.host_csr_from_params(p)
    for mode in ["bu", "do"]:
        bfs = dbfs.BFS(p, gpu_runtime, mode=mode, max_hubs=max_hubs)
        if max_hubs is not None:
            assert bfs.graph.nhubs <= max_hubs
        if max_hubs != 0:
            assert bfs.graph.nhubs > 0
        bfs.engine.set_option("bu_whole_units", whole)  # 64 / 16 words per wave (compacted hub kernel)
        bfs.engine.set_option("bu_small_waves", small)  # (split units: 4 words per wave on first levels)
        for src in bfs.sample_roots(3, seed=11):
            _check(bfs, csr, src)
        bfs.engine.set_option("device_loop", 0)
        _check(bfs, csr, bfs.sample_roots(1, seed=12)[0])


def test_full_scale_rmat20_gpu(gpu_runtime):
    """RMAT-20 at the default thresholds, exact against the CPU oracle: whole
    64-word units per wave chosen by occupancy (16 K units >= the resident wave
    slots), 2^19 hubs, deferred row scans, sparse and dense top-down levels."""
    p = dbfs.rmat_params(20, 16, 5)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, gpu_runtime, mode="do")
    assert bfs.graph.nhubs > 1 << 16
    dirs = set()
    for src in bfs.sample_roots(2, seed=21):
        res = _check(bfs, csr, src)
        dirs.update(lv["dir"] for lv in res.levels)
        assert bfs.validate(src)
    assert dirs == {"T", "B"}


def test_hub_lds_virtual_ranks_gpu():
    """Hub path on 3 virtual ranks: the hub frontier bits are gathered from the
    all-gathered global frontier of every rank."""
    p = dbfs.rmat_params(15, 16, 59)
    csr = dbfs.host_csr_from_params(p)
    srcs = [2, 900, 20000]
    exp = [dbfs.cpu_bfs(csr, s)[0] for s in srcs]

    def body(rt):
        bfs = dbfs.BFS(p, rt, mode="do", max_hubs=2000)
        assert 0 < bfs.graph.nhubs <= 2000
        out = []
        for s in srcs:
            bfs.run(s)
            out.append(bfs.levels())
        return out

    for rank_out in run_virtual_ranks(3, body, device="hip"):
        for lv, e in zip(rank_out, exp):
            assert np.array_equal(lv, e)


def test_multiprocess_ranks_share_one_gpu_tcp():
    """The one-process-per-rank launch (torch.distributed.run, as the driver
    runs bench.py on 8 GPUs) with 2 ranks on this one GPU: every rank runs the
    real HIP kernels on its shard; collectives go through the TCP communicator
    (RCCL refuses two ranks on one device).  The traversal must validate."""
    import json
    import socket
    import subprocess
    import sys

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, DBFS_DEVICE="0", DBFS_COMM="tcp")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"), "--gpus", "2", "--scale", "18",
           "--steps", "2", "--warmup", "1"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["n_gpus"] == 2 and rec["validated"] is True


def test_bench_self_spawned_ranks_share_one_gpu():
    """bench.py --gpus 2 WITHOUT a launcher (the parent spawns the rank
    processes itself, as when a driver runs `python bench.py --gpus 8`): both
    ranks run the HIP kernels on device 0, TCP collectives, every timed root
    validated, and the JSON reports the ranks the communicator formed."""
    import json
    import subprocess
    import sys

    env = dict(os.environ, DBFS_DEVICE="0", DBFS_COMM="tcp")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--scale", "18", "--steps", "3",
           "--warmup", "1"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["comm_ranks"] == 2 and rec["comm"] == "tcp"
    assert rec["devices"] == ["hip:0", "hip:0"]
    assert rec["validated"] is True and rec["validated_roots"] == "3/3"


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["td", "do"])
@pytest.mark.parametrize("sparse_edges", [0, 64, 1 << 16, 1 << 40])
def test_sparse_top_down_levels_gpu(gpu_runtime, mode, sparse_edges):
    """Sparse top-down levels (td_sparse_kernel: fetch-or claims, wave-
    aggregated packed append, last-workgroup level decision) interleaved with
    dense and bottom-up levels: hub root (> one edge block), 3000-level path,
    random blob; and RMAT-16 roots.  Same levels and records as the host loop."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from test_engine_cpu import _mixed_graph
    n, u, v = _mixed_graph()
    graphs = [(dbfs.build_csr(n, u, v), [0, 2999, 4500, 12345])]
    p = dbfs.rmat_params(16, 16, 47)
    csr = dbfs.host_csr_from_params(p)
    graphs.append((p, None))
    for g, roots in graphs:
        dev = dbfs.BFS(g, gpu_runtime, mode=mode)
        dev.engine.set_option("td_sparse_edges", sparse_edges)
        host = dbfs.BFS(g, gpu_runtime, mode=mode)
        host.engine.set_option("device_loop", 0)
        ref = g if roots is not None else csr
        for src in roots or dev.sample_roots(4, seed=9):
            a, b = dev.run(src), host.run(src)
            assert np.array_equal(dev.levels(), dbfs.cpu_bfs(ref, src)[0])
            strip = lambda r: [(l["dir"], l["frontier"], l["frontier_edges"], l["discovered"]) for l in r.levels]
            assert strip(a) == strip(b)
            assert (a.reached, a.edges, a.depth) == (b.reached, b.edges, b.depth)
            assert all(l["ms"] > 0 for l in a.levels)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["td", "bu", "do"])
def test_narrow_levels_gpu(gpu_runtime, mode):
    """One-byte levels (init_run uint4 fill, store_level in update / bottom-up /
    sparse kernels, widen_levels on read) equal the 32-bit path; a 700-level
    path overflows them and is rerun with 32-bit levels.  Nine roots cycle
    the per-run byte base (narrow_epochs) twice."""
    p = dbfs.rmat_params(16, 16, 13)
    csr = dbfs.host_csr_from_params(p)
    narrow, wide = dbfs.BFS(p, gpu_runtime, mode=mode), dbfs.BFS(p, gpu_runtime, mode=mode)
    wide.engine.set_option("narrow_levels", 0)
    for src in narrow.sample_roots(8, seed=4) + [17]:
        a, b = narrow.run(src), wide.run(src)
        assert np.array_equal(narrow.local_levels(), wide.local_levels())
        assert np.array_equal(narrow.levels(), dbfs.cpu_bfs(csr, src)[0])
        assert (a.reached, a.edges, a.depth) == (b.reached, b.edges, b.depth)
        assert narrow.validate(src)
    n = 700
    path = dbfs.build_csr(n, np.arange(n - 1), np.arange(1, n))
    deep = dbfs.BFS(path, gpu_runtime, mode=mode)
    for src in (0, 350):
        r = deep.run(src)
        assert np.array_equal(deep.levels(), np.abs(np.arange(n) - src))
        assert r.reached == n


@pytest.mark.gpu
def test_validator_counts_gpu(gpu_runtime):
    """Device Graph500 validator (thread-per-row, wave-per-long-row): clean
    levels give no violations; validating against another source flags exactly
    the two vertices whose level-0 status is wrong (RMAT hubs: rows > 64)."""
    p = dbfs.rmat_params(16, 16, 9)
    csr = dbfs.host_csr_from_params(p)
    assert int(np.diff(np.asarray(csr.row_off)).max()) > 64
    b = dbfs.BFS(p, gpu_runtime, mode="do")
    src, other = b.sample_roots(2, seed=8)
    b.run(src)
    assert list(b.engine.validate(int(src))) == [0, 0, 0]
    assert list(b.engine.validate(int(other))) == [0, 0, 2]


@pytest.mark.gpu
@pytest.mark.parametrize("vis_frac", [0.0, 0.75])
@pytest.mark.parametrize("mode", ["td", "do"])
def test_td_hub_filter_gpu(gpu_runtime, mode, vis_frac):
    """Top-down hub filter (hubs' visited bits in LDS, hub-encoded td_col) on
    every dense level (td_hub_edges=1), hub targets claimed through the hub
    marks + hub_apply: exact levels."""
    p = dbfs.rmat_params(17, 16, 21)
    csr = dbfs.host_csr_from_params(p)
    b = dbfs.BFS(p, gpu_runtime, mode=mode)
    b.engine.set_option("td_hub_edges", 1)
    b.engine.set_option("td_hub_vis_frac", vis_frac)
    b.engine.set_option("td_direct_edges", 1)
    for src in b.sample_roots(5, seed=3):
        r = b.run(src)
        exp = dbfs.cpu_bfs(csr, src)[0]
        assert np.array_equal(b.levels(), exp), src
        assert r.reached == int((exp != dbfs.UNREACHED).sum())
        assert b.validate(src)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["td", "bu", "do"])
def test_narrow_epochs_stale_bytes_gpu(gpu_runtime, mode):
    """Runs alternate between an RMAT component and a 62-level path (the
    deepest narrow traversal): each meets level bytes that the other component
    and earlier epochs left behind, which must read as unreached."""
    p = dbfs.rmat_params(14, 16, 3)
    rm = dbfs.host_csr_from_params(p)
    n0 = int(rm.n)
    deg = np.diff(np.asarray(rm.row_off))
    rows = np.repeat(np.arange(n0), deg)
    cols = np.asarray(rm.col)
    n1 = 63
    src_e = np.concatenate([rows, n0 + np.arange(n1 - 1)])
    dst_e = np.concatenate([cols, n0 + np.arange(1, n1)])
    csr = dbfs.build_csr(n0 + n1, src_e, dst_e)
    b = dbfs.BFS(csr, gpu_runtime, mode=mode)
    roots = np.nonzero(deg)[0][::997][:5].tolist()
    for i in range(10):
        src = roots[i // 2] if i % 2 == 0 else n0 + (0 if i % 4 == 1 else n1 - 1)
        r = b.run(src)
        exp = dbfs.cpu_bfs(csr, src)[0]
        assert np.array_equal(b.levels(), exp), (i, src)
        assert r.depth == int(exp[exp != dbfs.UNREACHED].max()) + 1


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["td", "bu", "do"])
def test_device_loop_several_ranks_gpu(gpu_runtime, mode):
    """Device loop with collectives in the level chains: RCCL (1 rank, forced
    exchange: the stream-ordered ncclAllGather / ncclAllToAll / ncclAllReduce
    between predicated kernels, level_finish on the reduced totals) and three
    virtual ranks on one GPU, against the host loop."""
    from distributed_cuda_bfs_amd.parallel.runtime import Runtime

    N = dbfs.native
    be = gpu_runtime.backend
    comm = N.nccl_comm(N.nccl_unique_id(), 0, 1, be)
    rt = Runtime(backend=be, comm=comm)
    p = dbfs.rmat_params(15, 16, 31)
    csr = dbfs.host_csr_from_params(p)
    strip = lambda r: [(l["dir"], l["frontier"], l["frontier_edges"], l["discovered"]) for l in r.levels]
    dev = dbfs.BFS(p, rt, mode=mode, force_exchange=True)
    dev.engine.set_option("td_byte_edges", 1 << 12)
    host = dbfs.BFS(p, rt, mode=mode, force_exchange=True)
    host.engine.set_option("device_loop", 0)
    for src in dev.sample_roots(3, seed=12):
        a, b = dev.run(src), host.run(src)
        assert np.array_equal(dev.levels(), dbfs.cpu_bfs(csr, src)[0])
        assert strip(a) == strip(b) and (a.reached, a.edges, a.depth) == (b.reached, b.edges, b.depth)
    comm.barrier()

    srcs = [5, 1234]

    def body(r):
        d, h = dbfs.BFS(p, r, mode=mode), dbfs.BFS(p, r, mode=mode)
        h.engine.set_option("device_loop", 0)
        out = []
        for s in srcs:
            x, y = d.run(s), h.run(s)
            out.append((d.levels(), strip(x) == strip(y)))
        return out

    for rank_out in run_virtual_ranks(3, body, device="hip"):
        for (lv, same), s in zip(rank_out, srcs):
            assert same and np.array_equal(lv, dbfs.cpu_bfs(csr, s)[0])


@pytest.mark.parametrize("mode,sparse_edges", [("bu", 0), ("td", 0), ("td", 1 << 16), ("do", 1 << 16)])
def test_back_to_back_runs_trailing_chain_gpu(gpu_runtime, mode, sparse_edges):
    """Runs issued back to back (the device loop ends without a synchronize,
    so the speculative chain enqueued after the last level -- bottom-up 'B',
    dense 'T' or sparse 'S' form -- is still in flight when the next run resets
    the mailbox): no stale stamp may leak into the next run.  Every run is
    compared with the CPU oracle, and its records with a fresh engine's."""
    p = dbfs.rmat_params(15, 16, 21)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, gpu_runtime, mode=mode)
    bfs.engine.set_option("td_sparse_edges", sparse_edges)
    roots = bfs.sample_roots(6, seed=4)
    results = [bfs.run(r) for r in roots]  # no synchronize in between
    for r, res in zip(roots, results):
        again = bfs.run(r)
        assert (res.reached, res.edges, res.depth) == (again.reached, again.edges, again.depth)
        exp, _ = dbfs.cpu_bfs(csr, r)
        assert np.array_equal(bfs.levels(), exp)


@pytest.mark.parametrize("knobs", [{}, {"list_cap_factor": 0.01}, {"list_form_edges": 0}])
def test_sparse_lists_several_ranks_gpu(gpu_runtime, knobs):
    """Several-rank device loop on the GPU kernels: sparse top-down chains
    (td_sparse claiming owned targets in place and appending remote ones to
    owner lists, the lists exchanged, td_sparse_apply settling them), dense
    chains when the lists are off or too small (re-enqueued), bottom-up
    chains fed by the previous level's fused gather + reduce -- one RCCL rank
    with the exchange forced and 3 / 8 virtual ranks, against the CPU oracle
    and the host loop."""
    from distributed_cuda_bfs_amd.parallel.runtime import Runtime

    N = dbfs.native
    be = gpu_runtime.backend
    comm = N.nccl_comm(N.nccl_unique_id(), 0, 1, be)
    rt = Runtime(backend=be, comm=comm)
    p = dbfs.rmat_params(16, 16, 37)
    csr = dbfs.host_csr_from_params(p)
    strip = lambda r: [(l["dir"], l["frontier"], l["frontier_edges"], l["discovered"]) for l in r.levels]
    dev = dbfs.BFS(p, rt, mode="do", force_exchange=True)
    for k, v in knobs.items():
        dev.engine.set_option(k, v)
    host = dbfs.BFS(p, rt, mode="do", force_exchange=True)
    host.engine.set_option("device_loop", 0)
    mis = 0
    for src in dev.sample_roots(4, seed=17):
        a, b = dev.run(src), host.run(src)
        mis += a.mispredicts
        assert np.array_equal(dev.levels(), dbfs.cpu_bfs(csr, src)[0])
        assert strip(a) == strip(b) and (a.reached, a.edges, a.depth) == (b.reached, b.edges, b.depth)
    if knobs.get("list_cap_factor", 1) < 1:
        assert mis > 0
    comm.barrier()

    srcs = [7, 4321, 60000]

    def body(r):
        d = dbfs.BFS(p, r, mode="do")
        for k, v in knobs.items():
            d.engine.set_option(k, v)
        return [(d.run(s), d.levels())[1] for s in srcs]

    for P in (3, 8):
        for rank_out in run_virtual_ranks(P, body, device="hip"):
            for lv, s in zip(rank_out, srcs):
                assert np.array_equal(lv, dbfs.cpu_bfs(csr, s)[0])


def test_peer_comm_two_ranks_share_one_gpu():
    """Peer-memory communicator: two self-spawned ranks on device 0 export
    their uncached windows over IPC, map each other's, pass the self-test
    (every collective with known patterns), then run the bench with the
    collectives as push / wait / unpack kernels; every timed root validated."""
    import json
    import subprocess
    import sys

    env = dict(os.environ, DBFS_DEVICE="0", DBFS_COMM="peer", DBFS_PEER_SLOT_MB="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--scale", "18", "--steps", "4",
           "--warmup", "1"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["comm"] == "peer+tcp" and rec["comm_note"] is None
    assert rec["validated"] is True and rec["validated_roots"] == "4/4"


@pytest.mark.parametrize("mode", ["td", "do"])
@pytest.mark.parametrize("direct_edges", [0, 1 << 16, 1 << 40])
def test_td_direct_levels_gpu(gpu_runtime, mode, direct_edges):
    """One rank, narrow levels: top-down levels store the level byte of every
    unvisited candidate directly (td_direct) from `direct_edges` frontier edges
    on (0: every dense level, 2^40: never); exact against the oracle, also
    with a long chain (levels past the narrow range fall back and rerun)."""
    p = dbfs.rmat_params(17, 16, 37)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, gpu_runtime, mode=mode)
    bfs.engine.set_option("td_direct_edges", direct_edges)
    for src in bfs.sample_roots(3, seed=41):
        _check(bfs, csr, src)
    n = 600
    chain = dbfs.build_csr(n, np.arange(n - 1, dtype=np.uint32), np.arange(1, n, dtype=np.uint32))
    cb = dbfs.BFS(chain, gpu_runtime, mode=mode)
    cb.engine.set_option("td_direct_edges", direct_edges)
    _check(cb, chain, 0)


@pytest.mark.parametrize("mode", ["td", "do"])
@pytest.mark.parametrize("bin_edges", [1, 1 << 20, 0])
def test_binned_top_down_gpu(gpu_runtime, mode, bin_edges):
    """One rank, binned top-down levels (targets binned by vertex range, one
    workgroup per bin claims them in LDS): every non-sparse top-down level (1),
    large ones only (2^20), none (0); exact against the oracle on RMAT and
    on a star whose centre's row spans many edge blocks."""
    p = dbfs.rmat_params(18, 16, 43)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, gpu_runtime, mode=mode)
    bfs.engine.set_option("td_bin_edges", bin_edges)
    bfs.engine.set_option("td_bin_min_rows", 0)  # (default: graphs of >= 2^26 vertices only)
    forms = set()
    for src in bfs.sample_roots(3, seed=47):
        res = _check(bfs, csr, src)
        forms.update(c[1] for c in res.chains)
    if bin_edges == 1:
        assert "X" in forms
    if bin_edges == 0:
        assert "X" not in forms
    n = 70000
    star = dbfs.build_csr(n, np.zeros(n - 1, dtype=np.uint32), np.arange(1, n, dtype=np.uint32))
    sb = dbfs.BFS(star, gpu_runtime, mode=mode)
    sb.engine.set_option("td_bin_edges", bin_edges)
    sb.engine.set_option("td_bin_min_rows", 0)
    _check(sb, star, 0)
    _check(sb, star, 5)


@pytest.mark.parametrize("mode", ["do", "td"])
def test_eight_virtual_ranks_rmat18_gpu(mode):
    """P = 8 virtual ranks on one GPU through the multi-rank device loop at
    RMAT-18: sparse (owner lists) and dense top-down chains, bottom-up levels
    fed by the fused gather + reduce; exact against the oracle and every chain
    form seen."""
    p = dbfs.rmat_params(18, 16, 61)
    csr = dbfs.host_csr_from_params(p)
    deg = np.diff(np.asarray(csr.row_off))
    hub = int(np.argmax(deg))
    reach = np.nonzero(dbfs.cpu_bfs(csr, hub)[0] != dbfs.UNREACHED)[0]
    srcs = [int(reach[len(reach) // 3]), int(reach[-1])]  # two roots in the giant component
    exp = [dbfs.cpu_bfs(csr, s)[0] for s in srcs]

    def body(rt):
        b = dbfs.BFS(p, rt, mode=mode)
        out, forms = [], set()
        for s in srcs:
            r = b.run(s)
            forms.update(c[1] for c in r.chains)
            out.append(b.levels())
        return out, forms

    for levels, forms in run_virtual_ranks(8, body, device="hip"):
        for got, e in zip(levels, exp):
            assert np.array_equal(got, e)
        assert "S" in forms and ("B" in forms if mode == "do" else "T" in forms)


def test_bottom_up_long_row_scanned_in_place_gpu(gpu_runtime):
    """A vertex with a 2^21-entry row whose only frontier neighbour sits at the
    end of its (hub-first) row: every bottom-up level scans the whole row in
    place (rows of >= 2^20 entries are not queued), and the level that reaches
    that neighbour finds it last."""
    p = dbfs.rmat_params(16, 16, 9)
    u0, v0 = (np.asarray(x, dtype=np.int64) for x in dbfs.generate_edges(p))
    n0 = p.n
    k = 1 << 21
    c = n0                                   # the star centre
    leaves = np.arange(n0 + 1, n0 + 1 + k, dtype=np.int64)
    # every leaf has degree 2 (the centre + a partner leaf), so the centre's
    # row is ordered by id; the last leaf's partner is RMAT vertex 5, the one
    # before it gets a pendant vertex instead
    partners = n0 + 1 + ((leaves - n0 - 1) ^ 1)
    partners[-1] = 5
    partners[-2] = n0 + 1 + k
    keep = (leaves < partners) | (np.arange(k) >= k - 2)
    u = np.concatenate([u0, np.full(k, c), leaves[keep]])
    v = np.concatenate([v0, leaves, partners[keep]])
    n = n0 + 2 + k
    csr = dbfs.build_csr(n, u.astype(np.uint32), v.astype(np.uint32))
    for mode in ["bu", "do"]:
        bfs = dbfs.BFS(csr, gpu_runtime, mode=mode)
        _check(bfs, csr, 5)
        _check(bfs, csr, 0)


@pytest.mark.parametrize("mode", ["do", "td"])
def test_td_fused_finish_gpu(gpu_runtime, mode):
    """td_fused_finish: the update's last workgroup finishes dense top-down
    levels; exact against the oracle."""
    p = dbfs.rmat_params(17, 16, 67)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, gpu_runtime, mode=mode)
    for src in bfs.sample_roots(3, seed=9):
        _check(bfs, csr, src)


@pytest.mark.parametrize("mode", ["do", "td"])
def test_run_many_gpu(gpu_runtime, mode):
    """run_many on the GPU: back-to-back device-loop traversals without a
    return to Python give the oracle's reach / depth per root, and the last
    run's levels exactly."""
    p = dbfs.rmat_params(17, 16, 29)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, gpu_runtime, mode=mode)
    srcs = bfs.sample_roots(6, seed=31)
    res = bfs.run_many(srcs)
    for r, s in zip(res, srcs):
        exp = dbfs.cpu_bfs(csr, s)[0]
        assert r.source == s
        assert r.reached == int(np.count_nonzero(exp != dbfs.UNREACHED))
        assert r.depth == int(exp[exp != dbfs.UNREACHED].max()) + 1
    assert np.array_equal(bfs.levels(), dbfs.cpu_bfs(csr, srcs[-1])[0])


def test_eight_virtual_ranks_rmat22_defaults_gpu():
    """P = 8 virtual ranks at RMAT-22 with the default thresholds: the shard
    (2^19 vertices) takes the 16-word bottom-up waves, the hubs are the full
    2^19, and the small top-down levels are sparse chains with owner lists; the
    levels equal the one-rank run's and the oracle's."""
    p = dbfs.rmat_params(22, 16, 3)
    csr = dbfs.host_csr_from_params(p)
    one = dbfs.BFS(p, init_runtime("hip"), mode="do")
    srcs = one.sample_roots(2, seed=11)
    exp = []
    for s in srcs:
        one.run(s)
        exp.append(one.levels())
    del one
    for s, e in zip(srcs, exp):
        assert np.array_equal(e, dbfs.cpu_bfs(csr, s)[0])

    def body(rt):
        b = dbfs.BFS(p, rt, mode="do")
        out, caps = [], []
        for s in srcs:
            r = b.run(s)
            caps += [c[2] for c in r.chains if c[1] == "S"]
            out.append(b.levels())
        return out, caps, b.graph.nhubs

    for levels, caps, nhubs in run_virtual_ranks(8, body, device="hip"):
        for got, e in zip(levels, exp):
            assert np.array_equal(got, e)
        assert caps  # sparse chains with owner lists at P = 8
        assert nhubs > 0


def _run_group(cmd, env, timeout):
    """Run a command that starts rank processes of its own (bench.py self-
    spawn) in a session of its own; past `timeout` the whole process group
    is killed (no orphaned rank keeps the GPU) and the test fails with the
    ranks' stderr tail -- what each rank logged last, and which collective
    a timed-out wait named."""
    import signal
    import subprocess

    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                         start_new_session=True)
    try:
        o, e = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)  # (the group this test started)
        o, e = p.communicate()
        pytest.fail(f"timed out after {timeout} s; stderr tail:\n{e[-6000:]}")
    return subprocess.CompletedProcess(cmd, p.returncode, o, e)


def test_peer_comm_four_ranks_share_one_gpu_rmat20():
    """Four self-spawned ranks on device 0 over the peer-memory transport at
    RMAT-20: every collective (gather + reduce, count-sized owner lists,
    candidate slices, pushed frontier slices) through the IPC windows; every
    timed root validated.  Ranks sharing a GPU run the collectives unfused and
    the direct exchanges' waits as one-wave launches (Comm::split_waits): a
    grid spinning in every workgroup could hold the CUs a co-resident rank's
    producer needs (the round-4 hang of this test)."""
    import json
    import sys

    env = dict(os.environ, DBFS_DEVICE="0", DBFS_COMM="peer", DBFS_PEER_SLOT_MB="16", DBFS_COMM_TIMEOUT_S="20")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", "4", "--scale", "20", "--steps", "4",
           "--warmup", "1", "--no-int32-pass", "--heldout-roots", "8", "--secondary", "none"]
    out = _run_group(cmd, env, 100)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["comm"] == "peer+tcp" and rec["n_gpus"] == 4
    assert rec["comm_direct"] is True  # (the direct exchanges passed their self-test on every rank)
    topo = rec["comm_topology"]
    assert topo["shared_device"] is True and topo["split_waits"] is True and topo["fused"] is False
    assert topo["peer_access"] == [[2] * 4] * 4 and topo["self_test"] == "ok"
    assert rec["validated"] is True and rec["validated_roots"] == "4/4"
    assert rec["heldout"]["validated_roots"] == "8/8"


def test_peer_comm_eight_ranks_share_one_gpu():
    """The driver's 8-rank shape over the peer-memory transport, rehearsed
    with eight self-spawned processes on device 0 (RMAT-19): the 16-peer
    tables, 8-way owner lists, pushed frontier slices and folded level ends
    at P = 8, every timed and held-out root validated."""
    import json
    import sys

    env = dict(os.environ, DBFS_DEVICE="0", DBFS_COMM="peer", DBFS_PEER_SLOT_MB="8", DBFS_PEER_FRONTIER_MB="2",
               DBFS_COMM_TIMEOUT_S="30")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", "8", "--scale", "19", "--steps", "4",
           "--warmup", "1", "--no-int32-pass", "--heldout-roots", "8", "--secondary", "none"]
    out = _run_group(cmd, env, 140)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["comm"] == "peer+tcp" and rec["n_gpus"] == 8 and rec["comm_direct"] is True
    topo = rec["comm_topology"]
    assert topo["shared_device"] is True and topo["self_test"] == "ok" and len(topo["peer_access"]) == 8
    assert rec["validated"] is True and rec["validated_roots"] == "4/4"
    assert rec["heldout"]["validated_roots"] == "8/8"


@pytest.mark.parametrize("ranks", [2, 4, 8])
def test_peer_fused_forms_share_one_gpu(ranks):
    """The separate-GPU forms of the peer transport -- every collective one
    fused launch, the direct exchanges' waits inside their consumer kernels
    (DBFS_PEER_SPLIT=0 keeps them on a shared GPU) -- the forms the first
    8-GPU run takes, with 2, 4 and 8 ranks on device 0.  Every grid whose
    workgroups all spin on a peer is sized for the co-resident ranks
    (Comm::coresident: the fused collectives' groups per peer, the owner
    side's grid), so no rank starves a peer's producer of CUs: every timed
    and held-out root validated."""
    import json
    import sys

    env = dict(os.environ, DBFS_DEVICE="0", DBFS_COMM="peer", DBFS_PEER_SLOT_MB="8", DBFS_PEER_FRONTIER_MB="2",
               DBFS_COMM_TIMEOUT_S="30", DBFS_PEER_SPLIT="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", str(ranks), "--scale", "19", "--steps",
           "4", "--warmup", "1", "--no-int32-pass", "--heldout-roots", "8", "--secondary", "none"]
    out = _run_group(cmd, env, 140)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    topo = rec["comm_topology"]
    assert topo["shared_device"] is True and topo["split_waits"] is False and topo["fused"] is True
    assert rec["validated_roots"] == "4/4" and rec["heldout"]["validated_roots"] == "8/8"
    assert rec["pushed_chains"] > 0


def test_peer_late_rank_completes():
    """A rank that publishes late: rank 1 sleeps 1.5 s before enqueueing level
    2 of every traversal (DBFS_FAULT_INJECT kind=delay) while its three peers'
    kernels of that level already wait for its exchanges on the device.  The
    traversals complete with every timed root validated, well inside the
    collective timeout (nothing spins in every workgroup of a grid)."""
    import json
    import sys

    env = dict(os.environ, DBFS_DEVICE="0", DBFS_COMM="peer", DBFS_PEER_SLOT_MB="16", DBFS_COMM_TIMEOUT_S="20",
               DBFS_FAULT_INJECT="rank=1,level=2,kind=delay,ms=1500")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", "4", "--scale", "18", "--steps", "3",
           "--warmup", "1", "--no-int32-pass", "--heldout-roots", "0", "--secondary", "none"]
    out = _run_group(cmd, env, 110)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["comm"] == "peer+tcp" and rec["validated_roots"] == "3/3"


def test_peer_hung_rank_names_the_stalled_collective():
    """A rank that never publishes (kind=hang at level 1): the peers' device
    waits give up after DBFS_COMM_TIMEOUT_S (5 s) and their error names the
    rank that timed out, the collective (sequence number, what it was, the
    level) and the rank it waited for -- an error well inside the test's
    limit, not a hang."""
    import subprocess
    import time

    port = _free_port_pair()
    procs = []
    for r in range(3):
        env = dict(os.environ, WORLD_SIZE="3", RANK=str(r), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port - 1), DBFS_BOOTSTRAP_PORT=str(port), DBFS_DEVICE="0", DBFS_COMM="peer",
                   DBFS_PEER_SLOT_MB="4", DBFS_COMM_TIMEOUT_S="5", DBFS_FAULT_INJECT="rank=1,level=1,kind=hang")
        procs.append(subprocess.Popen([os.path.join(REPO, "bin", "bfs"), "--rmat", "16", "5", "--no-oracle",
                                       "--quiet"], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    t0 = time.time()
    outs = {}
    for r in (0, 2):
        try:
            o, e = procs[r].communicate(timeout=60)
        except subprocess.TimeoutExpired:
            procs[r].kill()  # exact child PID
            o, e = procs[r].communicate()
        outs[r] = (procs[r].returncode, e)
    elapsed = time.time() - t0
    procs[1].kill()  # the hung rank (exact PID)
    procs[1].communicate()
    for r, (rc, e) in outs.items():
        assert rc != 0, e[-2000:]
        assert f"rank {r} timed out in collective #" in e and "waiting for rank 1" in e, e[-2000:]
        assert "level 1" in e, e[-2000:]
    assert elapsed < 50


@pytest.mark.parametrize("fault,comm", [("kind=rccl_init", "peer+tcp"), ("kind=peer_init,kind=rccl_init", "tcp"),
                                        ("kind=peer_init", "tcp")])
def test_transport_setup_failures_fall_back(fault, comm):
    """The multi-GPU setup does not depend on RCCL: with RCCL's setup forced
    to fail (DBFS_FAULT_INJECT kind=rccl_init) two ranks still form the peer
    transport over its TCP inner communicator and validate every timed root;
    with the peer windows' setup failing too, the RCCL fallback is tried
    (DBFS_TRY_RCCL=1: on a shared GPU too), fails on every rank, and the ranks
    agree on TCP; without DBFS_TRY_RCCL ranks sharing a GPU go straight to TCP
    (RCCL refuses -- or can hang in its setup with -- two ranks on one device)."""
    import json
    import sys

    env = dict(os.environ, DBFS_DEVICE="0", DBFS_COMM_TIMEOUT_S="20", DBFS_FAULT_INJECT=fault,
               DBFS_RCCL_INIT_TIMEOUT_S="10")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "DBFS_COMM", "DBFS_TRY_RCCL"):
        env.pop(k, None)
    if "rccl_init" in fault:
        env["DBFS_TRY_RCCL"] = "1"
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", "2", "--scale", "17", "--steps", "3",
           "--warmup", "1", "--no-int32-pass", "--heldout-roots", "0", "--secondary", "none"]
    out = _run_group(cmd, env, 110)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["comm"] == comm and rec["validated_roots"] == "3/3"
    if comm == "peer+tcp":
        assert rec["comm_topology"]["inner"] == "tcp" and rec["comm_inner_ops"] == 0


def _free_port_pair():
    import socket

    while True:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        if port < 65000:
            return port


def test_cli_peer_two_processes_share_one_gpu():
    """bin/bfs as two processes (WORLD_SIZE = 2, the reference's bfs_mpi.cu
    model) on device 0 over the peer-memory transport: IPC windows, TCP for
    what does not fit them (RCCL refuses a shared device); the reference's
    output lines, Output OK! against the oracle, Graph500 checks."""
    import json
    import subprocess

    port = _free_port_pair()
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port - 1), DBFS_BOOTSTRAP_PORT=str(port), DBFS_DEVICE="0", DBFS_COMM="peer",
                   DBFS_PEER_SLOT_MB="4", DBFS_COMM_TIMEOUT_S="60")
        procs.append(subprocess.Popen([os.path.join(REPO, "bin", "bfs"), "--rmat", "16", "5", "--validate", "--json"],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=110)
        except subprocess.TimeoutExpired:
            p.kill()  # exact child PID
            o, e = p.communicate()
        outs.append((p.returncode, o, e))
    for rc, o, e in outs:
        assert rc == 0, e[-3000:]
    o = outs[0][1]
    assert "Output OK!" in o and "Validation OK" in o
    rec = json.loads([l for l in o.splitlines() if l.startswith("{")][-1])
    assert rec["comm"] == "peer+tcp" and rec["ranks"] == 2


@pytest.mark.parametrize("gpus", [2, 4])
def test_cli_single_process_gpus_share_one_gpu(gpus):
    """The reference's own execution model -- one process driving P GPUs
    (bfs.cu:328-332, 577-609) -- as `bin/bfs --gpus P`, rehearsed on one GPU:
    DBFS_DEVICE pins every rank's backend to device 0 and defers its frees
    (Backend::set_deferred_frees), so the in-process peer transport runs with
    split waits between rank threads that share the device.  Levels equal the
    oracle ("Output OK!") and pass the Graph500 validator, several roots."""
    import json
    import subprocess

    env = dict(os.environ, DBFS_DEVICE="0", DBFS_COMM="peer", DBFS_PEER_SLOT_MB="4", DBFS_COMM_TIMEOUT_S="30")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    for src in ("5", "0"):
        out = subprocess.run([os.path.join(REPO, "bin", "bfs"), "--gpus", str(gpus), "--rmat", "17", src, "--validate",
                              "--json"], capture_output=True, text=True, timeout=110, env=env)
        assert out.returncode == 0, out.stderr[-3000:]
        assert "Output OK!" in out.stdout and "Validation OK" in out.stdout, out.stdout[-2000:]
        rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
        assert rec["ranks"] == gpus and rec["comm"].startswith("peer+"), rec


def test_cli_single_process_rccl_fallback_is_bounded():
    """The --gpus P path's RCCL fallback (ncclCommInitAll's work as a group of
    nonblocking inits, bounded by DBFS_RCCL_INIT_TIMEOUT_S): with the peer
    transport's setup failing (DBFS_FAULT_INJECT kind=peer_init) two ranks on
    device 0 either run over RCCL with exact levels or fail cleanly with an
    RCCL error -- within the bound, never a hang."""
    import subprocess
    import time

    env = dict(os.environ, DBFS_DEVICE="0", DBFS_FAULT_INJECT="kind=peer_init", DBFS_RCCL_INIT_TIMEOUT_S="20",
               DBFS_COMM_TIMEOUT_S="20")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    t0 = time.time()
    out = subprocess.run([os.path.join(REPO, "bin", "bfs"), "--gpus", "2", "--rmat", "14", "3"], capture_output=True,
                         text=True, timeout=100, env=env)
    elapsed = time.time() - t0
    assert elapsed < 80
    if out.returncode == 0:
        assert "Output OK!" in out.stdout
    else:
        assert "RCCL" in out.stderr, out.stderr[-2000:]


def test_in_process_peer_refuses_a_shared_device():
    """The in-process peer transport (GroupBootstrap, the --gpus P path: each
    rank's window shared as a device pointer) needs one device per rank:
    threads sharing a device cannot spin on each other's flags (a hipFree in
    one waits for the other's collective).  On one GPU every rank refuses,
    agreed, so every rank can fall back together."""
    import threading

    from distributed_cuda_bfs_amd._native import N
    from distributed_cuda_bfs_amd.parallel.runtime import make_backend

    P = 2
    group = N.VirtualGroup(P)
    errs = [None] * P

    def body(r):
        be = make_backend("hip", 0)
        inner = N.virtual_comm(group, r, be)
        try:
            N.peer_comm(N.group_bootstrap(group, r), be, inner, 1 << 20)
        except Exception as e:  # noqa: BLE001
            errs[r] = str(e)

    th = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    assert all(e and "share device" in e for e in errs), errs


def test_peer_direct_exchange_long_chain(tmp_path):
    """Two ranks on device 0 over the peer transport, on a 3000-vertex path
    with a few shortcuts: thousands of sparse levels, each one direct owner-list
    exchange (td_sparse -> the owner's window) and one level end folded into
    td_sparse_apply's last workgroup -- the tagged cells reused every two
    exchanges, workgroups of the apply that start after their level's end.
    Every timed root validated (device validator + totals of the timed run)."""
    import json
    import subprocess
    import sys

    n = 3000
    lines = [f"{i} {i + 1}" for i in range(n - 1)] + [f"{i} {i + 700}" for i in range(0, n - 700, 311)]
    path = tmp_path / "chain.txt"
    path.write_text(f"{n} {len(lines)}\n" + "\n".join(lines) + "\n")  # (the reference's header: n m)
    env = dict(os.environ, DBFS_DEVICE="0", DBFS_COMM="peer", DBFS_PEER_SLOT_MB="4", DBFS_COMM_TIMEOUT_S="30")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", "2", "--graph", str(path), "--steps", "3",
           "--warmup", "1", "--no-int32-pass"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["comm"] == "peer+tcp" and rec["comm_direct"] is True and rec["validated_roots"] == "3/3"


@pytest.mark.parametrize("bits", [1, 0])
def test_sparse_level_from_bitmap_gpu(gpu_runtime, bits):
    """td_sparse_bits: the sparse top-down level after a bottom-up one reads
    the bottom-up output bitmap (a wave per unit, edges from the wave's degree
    prefix, two-level ticket) instead of a compacted work list; exact against
    the oracle on one rank (RMAT-18, RMAT-20: 16-unit grids up to the 1024-
    workgroup cap) and on 3 virtual ranks (owner lists after it)."""
    for scale in (18, 20):
        p = dbfs.rmat_params(scale, 16, 71)
        csr = dbfs.host_csr_from_params(p)
        bfs = dbfs.BFS(p, gpu_runtime, mode="do")
        bfs.engine.set_option("td_sparse_bits", bits)
        forms = ""
        for src in bfs.sample_roots(3, seed=5):
            res = _check(bfs, csr, src)
            forms += "".join(c[1] for c in res.chains) + "|"
        assert "BS" in forms
    p = dbfs.rmat_params(17, 16, 71)
    csr = dbfs.host_csr_from_params(p)
    srcs = [int(s) for s in dbfs.BFS(p, gpu_runtime, mode="do").sample_roots(2, seed=8)]

    def body(rt):
        b = dbfs.BFS(p, rt, mode="do")
        b.engine.set_option("td_sparse_bits", bits)
        return [(b.run(s), b.levels())[1] for s in srcs]

    for rank_out in run_virtual_ranks(3, body, device="hip"):
        for lv, s in zip(rank_out, srcs):
            assert np.array_equal(lv, dbfs.cpu_bfs(csr, s)[0])



@pytest.mark.parametrize("P", [4, 8])
def test_shadow_replay_direct_gpu(P):
    """Shadow ranks on the GPU: rank r of a P-rank traversal (recorded over
    virtual ranks) replayed alone through the direct-exchange paths -- sparse
    levels' lists read in place, tiny levels fused into one launch
    (xfuse_edges), folded level ends -- computes the recorded levels."""
    from distributed_cuda_bfs_amd.parallel.shadow import shadow_ranks

    p = dbfs.rmat_params(17, 16, 5)
    runs = shadow_ranks(p, P, [0, P - 1], [3, 777, 40000], mode="do", device="hip")
    for s in runs:
        assert s.exact, (s.rank, s.levels, s.recorded_levels)


@pytest.mark.parametrize("whole", [1, -1])
@pytest.mark.parametrize("max_hubs", [500, 4000, None])
def test_hub_cut_bottom_up_gpu(gpu_runtime, max_hubs, whole):
    """Hub-cut first bottom-up levels (bu_cut_prep + the kCut hub kernel):
    the non-hub frontier's neighbours claimed top-down into the claim bitmap,
    rows scanned up to their first non-hub neighbour, claimed vertices merged
    into the output and their statistics -- exact against the oracle with the
    cut on every first bottom-up level (1 << 40), at the default bound, and
    off; bottom-up-only runs cut level 0 (the root's frontier); 32-bit levels
    keep the claims in a byte array of their own (kCutClaims)."""
    p = dbfs.rmat_params(18, 16, 61)
    csr = dbfs.host_csr_from_params(p)
    for mode, alpha, narrow in [("do", 24.0, 1), ("do", 2.0, 1), ("do", 1e9, 1), ("bu", 24.0, 1), ("do", 2.0, 0),
                                ("bu", 24.0, 0)]:
        bfs = dbfs.BFS(p, gpu_runtime, mode=mode, alpha=alpha, max_hubs=max_hubs)
        assert bfs.graph.nhubs > 0
        bfs.engine.set_option("bu_whole_units", whole)
        bfs.engine.set_option("narrow_levels", narrow)
        for cut in [None, 1 << 40, 0]:
            if cut is not None:
                bfs.engine.set_option("bu_cut_edges", cut)
            for src in bfs.sample_roots(2, seed=17):
                _check(bfs, csr, src)


def _bench_peer(args, timeout=200, **env_extra):
    import json
    import subprocess
    import sys

    env = dict(os.environ, DBFS_DEVICE="0", DBFS_COMM="peer", DBFS_COMM_TIMEOUT_S="60", **env_extra)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py")] + args + ["--heldout-roots", "0", "--secondary",
                                                                          "none", "--no-int32-pass"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])


@pytest.mark.parametrize("ranks", [2, 4])
def test_all_reached_stop_peer_ranks(ranks):
    """The all-reached stop with several ranks over the peer transport (direct
    owner lists and level ends, pushed frontiers): self-spawned ranks on device
    0 traverse a connected uniform graph of mean degree 28 in do mode, roots
    back to back.  The stop leaves the last frontier (and any pushed slice of
    it) unconsumed; every timed root is validated against the oracle, and the
    stop must have fired."""
    rec = _bench_peer(["--gpus", str(ranks), "--uniform", "262144:3670016", "--mode", "do", "--steps", "6",
                       "--warmup", "1"])
    assert rec["comm_direct"] is True and rec["validated_roots"] == "6/6"
    assert rec["all_reached_stops"] > 0


def test_peer_slot_rounds_build_and_ingest(tmp_path):
    """Collectives larger than a window slot go through the windows in
    slot-sized rounds (PeerComm::rounds), never to the wrapped transport: two
    ranks on device 0 with 64 KiB slots build RMAT-19 (the degree all-gather is
    1 MiB per rank: 16 rounds; the bottom-up gathers 1-2 rounds) and ingest an
    edge list whose per-pair volumes are skewed (rank 0's half of the file
    routes every entry to rank 1: an all-to-all-v of dozens of rounds one way,
    a few the other).  Every timed root validated; comm_inner_ops == 0."""
    rec = _bench_peer(["--gpus", "2", "--scale", "19", "--steps", "4", "--warmup", "1"], DBFS_PEER_SLOT_KB="64")
    assert rec["comm"] == "peer+tcp" and rec["validated_roots"] == "4/4"
    assert rec["comm_inner_ops"] == 0 and rec["comm_peer_ops"] > 0
    rng = np.random.default_rng(3)
    n, m = 200000, 400000
    half = m // 2
    u = np.concatenate([rng.integers(n // 2, n, half), rng.integers(0, n, m - half)])
    v = np.concatenate([rng.integers(n // 2, n, half), rng.integers(0, n, m - half)])
    path = tmp_path / "skew.txt"
    path.write_text(f"{n} {m}\n" + "".join(f"{a} {b}\n" for a, b in zip(u, v)))
    rec = _bench_peer(["--gpus", "2", "--graph", str(path), "--steps", "4", "--warmup", "1"],
                      DBFS_PEER_SLOT_KB="64")
    assert rec["validated_roots"] == "4/4" and rec["config"]["input_edges"] == m
    assert rec["comm_inner_ops"] == 0


_CUT = ["bu_cut_mf_frac=1", "bu_cut_edges=1099511627776"]


@pytest.mark.parametrize("opts", [["xfuse_edges=4096"], ["bu_merge_visited=0"],
                                  ["xfuse_edges=4096", "bu_merge_visited=0"],
                                  ["direct_frontier=0"], ["direct_frontier=0", "xfuse_edges=0"],
                                  _CUT, _CUT + ["narrow_levels=0"], _CUT + ["direct_frontier=0"]])
def test_peer_multirank_options(opts):
    """The multi-rank options -- tiny sparse levels fused into one launch
    (xfuse_edges), bottom-up levels without the visited merge of the gathered
    frontier (bu_merge_visited=0), the frontier gathered by the level end
    instead of pushed by the kernels (direct_frontier=0), and the hub cut
    forced on every first bottom-up level (its remote claims' all-to-all over
    the windows; 32-bit levels keep the claims in their own bytes) -- over the
    peer transport with 4 processes on device 0 at RMAT-18: every timed root
    validated (the forced cut: taken in the profiled traversal)."""
    args = ["--gpus", "4", "--scale", "18", "--steps", "6", "--warmup", "1"]
    for o in opts:
        args += ["--opt", o]
    rec = _bench_peer(args, DBFS_PEER_SLOT_MB="16")
    assert rec["comm_direct"] is True and rec["validated_roots"] == "6/6"
    if "bu_cut_mf_frac=1" in opts:
        assert rec["cut_chains"] > 0


@pytest.mark.parametrize("opts", [[], ["bu_merge_visited=1"]])
def test_peer_direct_frontier(opts):
    """Pushed frontier slices (EngineOptions::direct_frontier, the default with
    several ranks on the peer transport): the top-down
    update and bottom-up kernels store their output words into the peers'
    windows and the next bottom-up level's hub_gather copies them in (the level
    end carries only totals).  4 processes on device 0 at RMAT-18, every timed
    root validated, and the profiled traversal did push."""
    args = ["--gpus", "4", "--scale", "18", "--steps", "6", "--warmup", "1"]
    for o in opts:
        args += ["--opt", o]
    rec = _bench_peer(args, DBFS_PEER_SLOT_MB="16")
    assert rec["comm_direct"] is True and rec["validated_roots"] == "6/6"
    assert rec["pushed_chains"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("parts", [2, 4])
@pytest.mark.parametrize("mode", ["td", "do"])
@pytest.mark.parametrize("bits", [False, True])
def test_split_levels_gpu(gpu_runtime, parts, mode, bits):
    """Split top-down levels on the GPU (TdArgs::split_k: each part a run of
    the edge steps, refresh_visited between parts, the update forced): every
    direct top-down level split, levels exact against the oracle.  bits: the
    device picks the bitmap form for every level (td_direct_edges above the
    graph's edges, ctrl->bytes 0) -- the parts claim into `next` and the
    refreshes between them find no level bytes."""
    p = dbfs.rmat_params(18, 16, 23)
    csr = dbfs.host_csr_from_params(p)
    b = dbfs.BFS(p, gpu_runtime, mode=mode)
    if bits:
        b.engine.set_option("td_direct_edges", float(1 << 40))
    else:
        b.engine.set_heuristics(24.0, 24.0, 8, td_byte_edges=0)
    b.engine.set_option("td_split_edges", 1)
    b.engine.set_option("td_split_parts", parts)
    b.engine.set_option("td_sparse_edges", 0)
    used = False
    for s in b.sample_roots(4, seed=3):
        r = b.run(s)
        assert np.array_equal(b.levels(), dbfs.cpu_bfs(csr, s)[0]), s
        used = used or any(c[6] in (parts, 2 * parts) for c in r.chains)
    assert used


@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("mode", ["td", "do"])
def test_high_diameter_grid_gpu(P, mode):
    """The road-like 2-D grid (256 x 200: 454 levels from a corner, a few
    hundred vertices each): past the one-byte levels, hundreds of tiny
    sparse levels in a row through the device loop -- every one stamped and
    exact against the oracle, one rank and three virtual ranks."""
    p = dbfs.grid_params(256, 200)
    csr = dbfs.host_csr_from_params(p)
    srcs = [0, 256 * 100 + 128, 256 * 200 - 1, 0]
    exp = {s: dbfs.cpu_bfs(csr, s)[0] for s in set(srcs)}

    def body(rt):
        bfs = dbfs.BFS(p, rt, mode=mode)
        out = []
        for s in srcs:
            res = bfs.run(s)
            out.append((s, res, bfs.levels()))
        return out

    for rank_out in run_virtual_ranks(P, body, device="hip"):
        for s, res, lv in rank_out:
            assert np.array_equal(lv, exp[s]), _describe(s, res, lv, exp[s])
            assert res.depth == int(exp[s].max()) + 1
