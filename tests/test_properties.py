"""Fixture shapes and property tests on the CPU backend.

Shapes: chain, star, complete K8, two components, self-loops + duplicates,
isolated vertices, odd N / N not divisible by P.  Property: for random small
multigraphs, every mode on P virtual ranks gives exactly the oracle's levels
and a valid Graph500 parent tree.
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import distributed_cuda_bfs_amd as dbfs
from distributed_cuda_bfs_amd.parallel.runtime import init_runtime, run_virtual_ranks
from distributed_cuda_bfs_amd.utils.validate import parents_are_valid

MODES = list(dbfs.MODES)
U = dbfs.UNREACHED


@pytest.fixture(scope="module")
def rt():
    return init_runtime("cpu")


def _csr(n, edges):
    e = np.asarray(edges, dtype=np.uint32).reshape(-1, 2)
    return dbfs.build_csr(n, e[:, 0], e[:, 1])


def _all_modes(csr, src, rt):
    out = {}
    for mode in MODES:
        bfs = dbfs.BFS(csr, rt, mode=mode)
        bfs.run(src)
        out[mode] = bfs.levels()
    return out


def test_complete_k8(rt):
    csr = _csr(8, [(i, j) for i in range(8) for j in range(i + 1, 8)])
    for src in range(8):
        for mode, lv in _all_modes(csr, src, rt).items():
            exp = np.ones(8, dtype=np.int32)
            exp[src] = 0
            assert np.array_equal(lv, exp), mode


def test_star_center_and_leaf(rt):
    n = 101
    csr = _csr(n, [(0, i) for i in range(1, n)])
    for mode, lv in _all_modes(csr, 0, rt).items():
        assert lv[0] == 0 and (lv[1:] == 1).all(), mode
    for mode, lv in _all_modes(csr, 57, rt).items():
        assert lv[57] == 0 and lv[0] == 1 and (np.delete(lv, [0, 57]) == 2).all(), mode


def test_isolated_source_and_unreachable(rt):
    # vertices 5..9 isolated; two components {0,1,2} {3,4}
    csr = _csr(10, [(0, 1), (1, 2), (3, 4)])
    for mode, lv in _all_modes(csr, 7, rt).items():
        assert lv[7] == 0 and (np.delete(lv, 7) == U).all(), mode
    for mode, lv in _all_modes(csr, 4, rt).items():
        assert list(lv[:5]) == [U, U, U, 1, 0], mode


edge_lists = st.integers(min_value=1, max_value=70).flatmap(
    lambda n: st.tuples(
        st.just(n),
        st.lists(st.tuples(st.integers(0, n - 1), st.integers(0, n - 1)), min_size=0, max_size=4 * n),
        st.integers(0, n - 1),
    ))


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(edge_lists, st.sampled_from([1, 2, 3]), st.sampled_from(MODES))
def test_random_graphs_all_modes_virtual_ranks(data, P, mode):
    n, edges, src = data
    csr = _csr(n, edges if edges else np.zeros((0, 2)))
    exp = dbfs.cpu_bfs(csr, src)[0]

    def body(rt):
        bfs = dbfs.BFS(csr, rt, mode=mode)
        bfs.run(src)
        return bfs.levels(), bfs.parents(src)

    for lv, par in run_virtual_ranks(P, body, device="cpu"):
        assert np.array_equal(lv, exp)
        assert parents_are_valid(csr, lv, par, src)


@settings(max_examples=15, deadline=None)
@given(st.integers(6, 11), st.integers(1, 16), st.integers(0, 2**31 - 1))
def test_random_rmat_do_equals_oracle(scale, ef, seed):
    rt = init_runtime("cpu")
    p = dbfs.rmat_params(scale, ef, seed)
    csr = dbfs.host_csr_from_params(p)
    bfs = dbfs.BFS(p, rt, mode="do")
    for src in bfs.sample_roots(2, seed=seed % 97):
        bfs.run(src)
        assert np.array_equal(bfs.levels(), dbfs.cpu_bfs(csr, src)[0])
