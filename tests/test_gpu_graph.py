"""Device graph inputs (csrc/ge_graph.hip) against the host generators
(ge_rmat_csr / ge_largest_component in csrc/ge_host.cpp, whose R-MAT definition
tests/graphs.py restates): the same CSR arrays, bit for bit.  The reference's
LCC step is examples/embedder.cpp:35-93 (its R-MAT input is synthetic here, as
SURVEY.md 8(d) specifies)."""
import numpy as np
import pytest

import ge_amd as ge
import graphs as G

pytestmark = pytest.mark.gpu


def _same(a, b):
    return all(np.array_equal(x, y) for x, y in zip(a, b))


@pytest.mark.parametrize("n,draws,seed", [(2, 5, 1), (37, 200, 3), (1000, 8000, 12345),
                                          (4096, 40000, 7), (100_000, 900_000, 5)])
def test_rmat_device_matches_host(ctx, n, draws, seed):
    assert _same(ctx.rmat_csr(n, draws, seed=seed), ge.rmat_csr(n, draws, seed=seed))
    assert _same(ctx.rmat_csr(n, draws, seed=seed, lcc=True),
                 ge.largest_component(ge.rmat_csr(n, draws, seed=seed)))
    if n <= 4096:  # the numpy definition
        assert _same(ctx.rmat_csr(n, draws, seed=seed), G.rmat(n, draws, seed=seed))


def test_lcc_device_ties_and_components(ctx):
    """Several components of equal largest size (the first one -- smallest vertex
    -- wins), isolated vertices, weights carried over."""
    import scipy.sparse as sp
    edges = [(5, 9), (9, 2), (2, 5), (0, 7), (7, 3), (3, 0), (11, 12), (13, 14), (14, 15)]
    r = [a for a, b in edges] + [b for a, b in edges]
    c = [b for a, b in edges] + [a for a, b in edges]
    w = np.arange(1, len(r) + 1, dtype=np.float64)
    M = sp.csr_matrix((w, (r, c)), shape=(17, 17))
    M.sort_indices()
    A = (M.indptr.astype(np.int32), M.indices.astype(np.int32), M.data)
    assert _same(ctx.largest_component(A), ge.largest_component(A))
    B = G.erdos_renyi(3000, 0.0006, seed=3)  # many small components
    assert _same(ctx.largest_component(B), ge.largest_component(B))


def test_c4_graph_device_matches_host(ctx):
    """configs[3]'s input (10M ids, 80M draws) and its LCC."""
    assert _same(ctx.rmat_csr(10_000_000, 80_000_000, seed=12345, lcc=True),
                 ge.largest_component(ge.rmat_csr(10_000_000, 80_000_000, seed=12345)))
