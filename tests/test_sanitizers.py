"""Host sanitizers: bin/bfs_asan is the CLI with every host
translation unit built with AddressSanitizer + UndefinedBehaviorSanitizer
(`make asan`).  GPU sanitizers are unavailable on this pool, so the runs use
the CPU backend; they cover the engine, partitioning, communicators (virtual
threads and multi-process TCP), graph I/O and the error paths."""
import os
import socket
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_BIN = os.path.join(REPO, "bin", "bfs_asan")
DATA = os.path.join(REPO, "tests", "data")


@pytest.fixture(scope="module")
def asan_bin():
    # (pytest-xdist workers each run this fixture: serialise the build)
    import fcntl
    os.makedirs(os.path.join(REPO, "build-asan"), exist_ok=True)
    with open(os.path.join(REPO, "build-asan", ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        out = subprocess.run(["make", "-j8", "asan"], cwd=REPO, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    return ASAN_BIN


def _env(**kw):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=24")
    env.update(kw)
    return env


def _run(binary, args, **kw):
    out = subprocess.run([binary] + args, capture_output=True, text=True, timeout=300, env=_env(**kw))
    assert "AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr, out.stderr[-4000:]
    return out


@pytest.mark.parametrize("mode", ["do", "td", "bu", "ref", "simple", "scan"])
def test_asan_modes_virtual_ranks(asan_bin, mode):
    out = _run(asan_bin, ["--rmat", "11", "3", "--cpu", "--virtual-ranks", "3", "--validate", "--mode", mode,
                          "--quiet"])
    assert out.returncode == 0, out.stderr[-4000:]


def test_asan_file_inputs_and_outputs(asan_bin, tmp_path):
    for f in ["chain8.txt", "dup_self.mtx", "two_components.txt"]:
        out = _run(asan_bin, ["0", os.path.join(DATA, f), "--cpu", "--levels-out", str(tmp_path / "lv.txt"),
                              "--cache", str(tmp_path / "g.csr")])
        assert out.returncode == 0, out.stderr[-4000:]
        out = _run(asan_bin, ["0", str(tmp_path / "g.csr"), "--cpu", "--roots", "3", "--json", "--quiet"])
        assert out.returncode == 0, out.stderr[-4000:]


def test_asan_error_paths(asan_bin, tmp_path):
    bad = tmp_path / "bad.txt"
    bad.write_text("3 2\n0 1\n1 7\n")  # vertex id out of range
    out = _run(asan_bin, ["0", str(bad), "--cpu"])
    assert out.returncode != 0
    out = _run(asan_bin, ["--rmat", "10", "3", "--cpu", "--virtual-ranks", "3", "--quiet"],
               DBFS_FAULT_INJECT="rank=2,level=1")
    assert out.returncode != 0 and "injected fault" in out.stderr


def test_asan_multiprocess_tcp(asan_bin):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(2):
        env = _env(WORLD_SIZE="2", RANK=str(r), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   DBFS_BOOTSTRAP_PORT=str(port))
        procs.append(subprocess.Popen([asan_bin, "--rmat", "10", "3", "--cpu", "--validate", "--quiet"], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    for p in procs:
        o, e = p.communicate(timeout=300)
        assert p.returncode == 0 and "AddressSanitizer" not in e, e[-4000:]
