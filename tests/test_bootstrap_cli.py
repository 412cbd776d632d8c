"""TCP bootstrap (RCCL unique-id exchange), the reference-compatible CLI, and
the bench.py output contract -- all on CPU."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BFS_BIN = os.path.join(REPO, "bin", "bfs")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _boot_worker(rank, world, port, q):
    import distributed_cuda_bfs_amd as dbfs

    b = dbfs.native.TcpBootstrap("127.0.0.1", port, rank, world, 60.0)
    got = b.broadcast(b"uid-128-bytes" if rank == 0 else b"")
    gathered = b.allgather(f"r{rank}".encode())
    b.barrier()
    q.put((rank, got, gathered))


def test_tcp_bootstrap_three_ranks():
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_boot_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=60) for _ in range(3)]
    for p in ps:
        p.join(timeout=30)
    for rank, got, gathered in outs:
        assert got == b"uid-128-bytes"
        assert gathered == [b"r0", b"r1", b"r2"]


def test_tcp_bootstrap_rejects_stray_connection():
    """A connection that does not speak the bootstrap handshake is dropped;
    the real ranks still form the group (any host could inject a
    fake peer or announce a huge message)."""
    import multiprocessing as mp
    import time

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    root = ctx.Process(target=_boot_worker, args=(0, 2, port, q))
    root.start()
    stray = None
    for _ in range(200):
        try:
            stray = socket.create_connection(("127.0.0.1", port), timeout=1)
            break
        except OSError:
            time.sleep(0.05)
    assert stray is not None
    stray.sendall(b"\xff" * 8 + b"\x01\x00\x00\x00")  # wrong magic, then a plausible rank
    stray.close()
    peer = ctx.Process(target=_boot_worker, args=(1, 2, port, q))
    peer.start()
    outs = sorted([q.get(timeout=60) for _ in range(2)])
    root.join(timeout=30)
    peer.join(timeout=30)
    assert [o[2] for o in outs] == [[b"r0", b"r1"]] * 2


def _run(args, **kw):
    return subprocess.run([BFS_BIN] + args, capture_output=True, text=True, timeout=120, **kw)


def test_cli_reference_stdout(data_dir):
    path = os.path.join(data_dir, "chain8.txt")
    out = _run(["0", path, "--cpu"])
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()
    # SURVEY Appendix A line set, in order (GPU-only peer-access line omitted on --cpu)
    expect_prefix = [path, "nodes num: 8", "edge num: 7", "finish load graph", "Number of vertices 8",
                     "Number of edges 14", "", "Starting sequential bfs."]
    assert lines[:8] == expect_prefix
    assert lines[8].startswith("Elapsed time in milliseconds : ") and lines[8].endswith(" ms.")
    assert "Starting queue parallel bfs." in lines
    assert out.stdout.endswith("Output OK!\n\n")  # bfs.cu:383 prints a trailing blank line


def test_cli_levels_out_and_json(tmp_path, data_dir):
    lv = tmp_path / "levels.txt"
    out = _run(["3", os.path.join(data_dir, "two_components.txt"), "--cpu", "--quiet", "--json",
                "--levels-out", str(lv), "--validate"])
    assert out.returncode == 0, out.stderr
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["reached"] == 3 and rec["edges"] == 3
    assert lv.read_text().split() == ["2147483647"] * 3 + ["0", "1", "2"] + ["2147483647"] * 4


@pytest.mark.parametrize("mode", ["ref", "td", "bu", "do", "simple"])
def test_cli_modes_rmat_virtual(mode):
    out = _run(["--rmat", "10", "5", "--cpu", "--mode", mode, "--virtual-ranks", "3", "--quiet", "--validate"])
    assert out.returncode == 0, out.stdout + out.stderr


def test_cli_errors(tmp_path):
    out = _run(["0", str(tmp_path / "nope.txt"), "--cpu"])
    assert out.returncode != 0 and "not open" in out.stderr
    out = _run(["0"])
    assert out.returncode == 2
    bad = tmp_path / "g.txt"
    bad.write_text("2 1\n0 1\n")
    out = _run(["5", str(bad), "--cpu", "--quiet"])
    assert out.returncode != 0 and "out of range" in out.stderr


def test_cli_roots_and_cache(tmp_path):
    cache = tmp_path / "g.csr"
    out = _run(["--rmat", "9", "0", "--cpu", "--quiet", "--cache", str(cache), "--roots", "3"])
    assert out.returncode == 0, out.stderr
    assert "harmonic-mean GTEPS" in out.stdout
    out = _run(["0", str(cache), "--cpu", "--quiet"])
    assert out.returncode == 0, out.stderr


def test_bench_contract_cpu():
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--device", "cpu", "--scale", "10",
                          "--steps", "3", "--warmup", "1"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in rec
    assert rec["steps"] == 3 and rec["warmup"] == 1 and rec["n_gpus"] == 1
    assert rec["value"] > 0 and rec["validated"] is True
    for k in ("model", "global_batch", "seq_len", "parallelism"):
        assert k in rec["config"]
    # honesty fields: what the timed kernels wrote, and the validated roots
    # are the timed ones (totals cross-checked against the timed traversal)
    assert rec["level_state_dtype"] in ("uint8", "int32")
    assert rec["dtype"] == ("uint8 levels (int32 on read)" if rec["level_state_dtype"] == "uint8" else "int32")
    assert rec["validated_roots"] == "3/3" and rec["primary"] is None
    assert rec["value"] == pytest.approx(rec["traversed_edges_mean"] * 3 / (rec["ms_per_step"] * 3 * 1e6), rel=1e-2)


def test_bench_self_spawn_cpu():
    """``bench.py --gpus 3`` without a launcher starts 3 rank processes itself
    (no torchrun): one JSON line from rank 0, the communicator really formed 3
    ranks, every timed root validated, honesty fields present."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "3", "--device", "cpu",
                          "--scale", "10", "--steps", "3", "--warmup", "1"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 3 and rec["comm_ranks"] == 3 and rec["comm"] == "tcp"
    assert rec["devices"] == ["cpu:-1"] * 3
    assert rec["validated"] is True and rec["validated_roots"] == "3/3"
    assert rec["level_state_dtype"] == "uint8" and rec["value_int32_levels"] > 0
    assert rec["config"]["parallelism"] == "1d-vertex-partition x3"


def test_bench_self_spawn_failure_propagates():
    """A failing rank makes the self-spawned job fail (no hang, non-zero exit)."""
    env = dict(os.environ, DBFS_FAULT_INJECT="rank=1,level=1,kind=exit", DBFS_COMM_TIMEOUT_S="20")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--device", "cpu",
                          "--scale", "9", "--steps", "2", "--warmup", "1"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode != 0
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


def test_bench_weak_scaling_cpu():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--device", "cpu",
                          "--scale", "9", "--weak", "--steps", "2", "--warmup", "1", "--no-int32-pass"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["scaling"] == "weak" and rec["config"]["vertices"] == 1 << 10
    assert rec["value_int32_levels"] is None


def test_bench_graph_file_cpu(tmp_path):
    # bench on a real graph file (the soc-LiveJournal1 / Friendster path;
    # here a small random edge list in the reference's `n m` + `u v` format)
    rng = np.random.default_rng(5)
    n, m = 2000, 12000
    path = tmp_path / "g.txt"
    e = rng.integers(0, n, size=(m, 2))
    path.write_text(f"{n} {m}\n" + "".join(f"{u} {v}\n" for u, v in e))
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--device", "cpu", "--graph", str(path),
                          "--steps", "3", "--warmup", "1"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert rec["config"]["model"] == "g.txt" and rec["config"]["vertices"] == n
    assert rec["config"]["input_edges"] == m and rec["validated"] is True
    assert rec["data"].startswith("file g.txt") and rec["vs_baseline"] is None


def test_bench_uniform_graph_cpu():
    # --uniform N:M: a uniform-random graph generated like RMAT (the
    # soc-LiveJournal1-sized stand-in without the 1 GB text file); no RMAT
    # baseline applies to it
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--device", "cpu", "--uniform", "3001:20000",
                          "--mode", "td", "--steps", "2", "--warmup", "1", "--no-int32-pass"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["config"]["vertices"] == 3001 and rec["config"]["input_edges"] == 20000
    assert rec["data"].startswith("synthetic (uniform") and rec["vs_baseline"] is None
    assert rec["validated"] is True


@pytest.mark.parametrize("nproc,mode", [(2, "do"), (3, "ref")])
def test_bench_torchrun_multiprocess_cpu(nproc, mode):
    """The driver's N>1 launch (torch.distributed.run, one process per rank,
    127.0.0.1 rendezvous) on the CPU backend: bootstrap + TCP collectives +
    rank-0-only JSON line."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
           "--gpus", str(nproc), "--device", "cpu", "--scale", "10", "--steps", "2", "--warmup", "1",
           "--mode", mode]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == nproc and rec["validated"] is True
    assert rec["config"]["parallelism"] == f"1d-vertex-partition x{nproc}"


def test_cli_level_csv(tmp_path):
    csv_path = tmp_path / "levels.csv"
    out = _run(["--rmat", "10", "3", "--cpu", "--quiet", "--roots", "3", "--json", "--phase-timing",
                "--level-csv", str(csv_path)])
    assert out.returncode == 0, out.stderr
    recs = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    rows = csv_path.read_text().strip().splitlines()
    assert rows[0] == "root,level,dir,frontier,frontier_edges,discovered,ms,run_ms"
    assert len(rows) - 1 == sum(len(r["levels"]) for r in recs)
    first = rows[1].split(",")
    assert int(first[0]) == recs[0]["source"] and first[1] == "0" and first[2] in "TB"


def test_cli_sharded_ingest_three_processes(tmp_path):
    """bin/bfs as 3 processes (WORLD_SIZE = 3, TCP, CPU backend) on an edge
    list: every rank parses only its own byte range of the file (the ranges
    tile the body, each rank reads about a third of the edges) and builds its
    shard from the edges routed to it -- unlike the reference, where every
    rank reads the whole file (bfs_mpi.cu:815).  Only the leader reads the
    file whole, for the CPU oracle: Output OK!, and the Graph500 checks pass."""
    rng = np.random.default_rng(11)
    n, m = 5000, 40000
    e = rng.integers(0, n, size=(m, 2))
    path = tmp_path / "g.txt"
    path.write_text(f"{n} {m}\n" + "".join(f"{u} {v}\n" for u, v in e))
    size = path.stat().st_size
    port = _free_port()
    procs = []
    for r in range(3):
        env = dict(os.environ, WORLD_SIZE="3", RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port - 1), DBFS_BOOTSTRAP_PORT=str(port), DBFS_COMM_TIMEOUT_S="60")
        procs.append(subprocess.Popen([BFS_BIN, "7", str(path), "--cpu", "--json", "--validate"], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, err = p.communicate(timeout=120)
        except subprocess.TimeoutExpired:
            p.kill()  # exact child PID
            o, err = p.communicate()
        outs.append((p.returncode, o, err))
    for rc, o, err in outs:
        assert rc == 0, err[-3000:]
    o = outs[0][1]
    lines = o.splitlines()
    assert lines[:6] == [str(path), f"nodes num: {n}", f"edge num: {m}", "finish load graph",
                         f"Number of vertices {n}", f"Number of edges {2 * m}"]
    assert "Output OK!" in o and "Validation OK" in o
    assert not outs[1][1].strip() and not outs[2][1].strip()  # (the leader prints)
    rec = json.loads([l for l in lines if l.startswith("{")][-1])
    ing = rec["ingest"]
    assert len(ing) == 3 and rec["ranks"] == 3
    assert len(f"{n} {m}") <= ing[0][0] <= len(f"{n} {m}\n") and ing[-1][1] == size
    for (b0, e0, _), (b1, _, _) in zip(ing, ing[1:]):
        assert e0 == b1 and b0 < e0  # contiguous, disjoint byte ranges
    assert sum(x[2] for x in ing) == m
    assert all(abs(x[2] - m / 3) < m / 10 for x in ing)  # about a third each


def test_cli_sharded_ingest_virtual_ranks_mtx(data_dir):
    """--virtual-ranks with a MatrixMarket file: sharded read (lines cut at
    line starts), levels equal the oracle's."""
    out = _run(["0", os.path.join(data_dir, "dup_self.mtx"), "--cpu", "--virtual-ranks", "2", "--json"])
    assert out.returncode == 0, out.stderr
    assert "Output OK!" in out.stdout
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert len(rec["ingest"]) == 2
