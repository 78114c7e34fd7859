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


# repel = 1e299 puts every pair outside the shared-reciprocal domain (the `/`
# path), and the self pair's cij / eps^2 overflows to inf: the reference skips
# j == i (include/forceatlas.hpp:151), so the kernels must too (a 0 * inf term
# would turn the row's sum into NaN).  One iteration stays finite.
HUGE_REPEL = 1e299


@pytest.mark.gpu
@pytest.mark.parametrize("n,env", [
    (40, {"GE_SMALL_MAX": "512"}),                         # one workgroup
    (300, {"GE_SMALL_MAX": "0"}),                          # fa_grouped_step
    (4000, {}),                                            # fa_grouped_stream
    (3000, {"GE_STREAM_MAX": "0", "GE_SMALL_MAX": "0"}),   # fa_repulse_strict + rows
])
def test_fa_self_pair_overflow(ctx, oracle, monkeypatch, n, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    A = G.rmat(n, 4 * n, seed=n)
    X0 = G.random_coords(n, 3, seed=1)
    want = oracle.force_atlas(A, 3, coords=X0, iterations=1, repel=HUGE_REPEL)
    got = ctx.force_atlas(A, 3, coords=X0, iterations=1, repel=HUGE_REPEL)
    assert np.isfinite(want).all()
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("sym", ["1", "0"])
def test_faml_self_pair_overflow(ctx, oracle, monkeypatch, sym):
    """Multilevel: resident packs, the symmetric kernel's diagonal tiles and row
    blocks, and the ordered-pair streamed kernel, all on the `/` path."""
    monkeypatch.setenv("GE_FAML_SYM", sym)
    sizes = [2600, 700, 257, 90, 5, 1]
    n = sum(sizes)
    A = G.submatrix(G.rmat(n, 6 * n, seed=2), np.arange(n))
    ip = np.cumsum([0] + sizes).astype(np.int32)
    PT = (ip, np.arange(n, dtype=np.int32))
    vA = ge.vertex_of(PT)
    m = len(sizes)
    cA = G.random_coords(m, 3, seed=m)
    rA = np.random.RandomState(m).uniform(0.1, 0.6, m)
    want = oracle.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=1, seed=3, repel=HUGE_REPEL)
    got = ctx.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=1, seed=3, repel=HUGE_REPEL)
    assert np.isfinite(want).all()
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_fa_flat_dimension_signed_zeros(ctx, oracle):
    """Every vertex has the same third coordinate: every repulsion and attraction
    term of that dimension is +-0, so the sums depend on starting from +0."""
    n = 2000
    A = G.rmat(n, 5 * n, seed=9)
    X0 = G.random_coords(n, 3, seed=4)
    X0[:, 2] = 0.0
    want = oracle.force_atlas(A, 3, coords=X0, iterations=5)
    got = ctx.force_atlas(A, 3, coords=X0, iterations=5)
    assert np.array_equal(got, want)
