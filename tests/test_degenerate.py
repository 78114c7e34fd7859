"""Degenerate inputs: one vertex, no edges, a single edge, several components,
and levels whose row tiles hold no entries.  The host partition is compared
with the oracle on the CPU; ForceAtlas, P^T A P and embed run on the device
(gpu marker) and must match the oracle bit for bit.

The reference has no tests for these; the expected results are
the oracle's restatement of include/forceatlas.hpp:89-574 and
src/partitioner.cpp:1550-1893, so they are pinned to the oracle only.
"""
import numpy as np
import pytest
import scipy.sparse as sp

import ge_amd as ge
import graphs as G


def csr(n, edges, w=1.0):
    if edges:
        r = [a for a, b in edges] + [b for a, b in edges]
        c = [b for a, b in edges] + [a for a, b in edges]
        M = sp.csr_matrix((np.full(len(r), w), (r, c)), shape=(n, n))
    else:
        M = sp.csr_matrix((n, n))
    M.sort_indices()
    return (M.indptr.astype(np.int32), M.indices.astype(np.int32), M.data.astype(np.float64))


CASES = {
    "one_vertex": csr(1, []),
    "one_edge": csr(2, [(0, 1)]),
    "no_edges": csr(5, []),
    "path3": csr(3, [(0, 1), (1, 2)]),
    "two_components": csr(6, [(0, 1), (1, 2), (3, 4)]),
    "star": csr(40, [(0, j) for j in range(1, 40)], w=2.5),
}


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("cf", [0.5, 0.1])
def test_partition_degenerate(oracle, name, cf):
    A = CASES[name]
    h = ge.partition(A, cf)
    want = oracle.partition(A, cf)
    assert len(h) == len(want)
    for a, b in zip(h, want):
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("small_max", ["512", "0"])  # one workgroup / grouped kernels
def test_fa_degenerate(ctx, oracle, monkeypatch, name, small_max):
    monkeypatch.setenv("GE_SMALL_MAX", small_max)
    A = CASES[name]
    n = len(A[0]) - 1
    X0 = G.random_coords(n, 3, seed=n)
    want = oracle.force_atlas(A, 3, coords=X0, iterations=25)
    got = ctx.force_atlas(A, 3, coords=X0, iterations=25)
    assert np.array_equal(got, want)
    assert np.isfinite(got).all()


@pytest.mark.gpu
@pytest.mark.parametrize("segments", ["1", "0"])
def test_fa_large_level_empty_tiles(ctx, oracle, monkeypatch, segments):
    """Large-level kernels (row tiles forced on) where most tiles hold no
    entries at all and the only edges form one heavy hub row (segments or
    the whole-row path), plus an edgeless level."""
    monkeypatch.setenv("GE_STREAM_MAX", "0")
    monkeypatch.setenv("GE_ROWS_TILES", "1")
    monkeypatch.setenv("GE_ROWS_SEGMENTS", segments)
    n = 3000
    for A in (csr(n, []), csr(n, [(7, j) for j in range(n) if j != 7 and j % 2 == 0])):
        X0 = G.random_coords(n, 3, seed=3)
        want = oracle.force_atlas(A, 3, coords=X0, iterations=3)
        assert np.array_equal(ctx.force_atlas(A, 3, coords=X0, iterations=3), want)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["one_edge", "no_edges", "two_components", "star"])
def test_ptap_and_embed_degenerate(ctx, oracle, name):
    A = CASES[name]
    hier = ge.partition(A, 0.5)
    As = [A]
    for PT in hier:
        C = ctx.ptap(As[-1], PT)
        for a, b in zip(C, oracle.ptap(As[-1], PT)):
            assert np.array_equal(a, b)
        As.append(C)
    X = ctx.embed(As, hier, 2, seed=5, base_iterations=2000, ml_iterations=50)
    want = oracle.embed(As, hier, 2, seed=5, base_iterations=2000, ml_iterations=50)
    assert np.array_equal(X, want)
