"""Radius ("kinetic ball") step on the device (csrc/ge_radius.hip) against the
oracle's serial event loop (oracle/ge_oracle.cpp orc_radius_step, restating
src/embed.cpp:615-777): r_A and the rescaled coordinates bit for bit.  Covers
the all-pairs base case, every level of R-MAT hierarchies (groups from 1
member to hubs), a star group (one pop, then every leaf at once), a path group
(one pop per round) and coincident coordinates (zero distance: the host loop
runs instead)."""
import ctypes

import numpy as np
import pytest

import ge_amd as ge
import graphs as G

pytestmark = pytest.mark.gpu


def _oracle_radius(oracle, cA, dim, base, PTc=None, cAc=None, rAc=None, Ac=None):
    m = cA.shape[0]
    cc = np.ascontiguousarray(cA.copy()).reshape(-1)
    rr = np.zeros(m)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    if base:
        oracle.lib().orc_radius_step(m, cc, rr, dim, 1, 0, None, None, None, None,
                                     np.zeros(1, np.int32), np.zeros(1, np.int32))
    else:
        pip = np.ascontiguousarray(PTc[0], np.int32)
        pix = np.ascontiguousarray(PTc[1], np.int32)
        cAc = np.ascontiguousarray(cAc)
        rAc = np.ascontiguousarray(rAc)
        oracle.lib().orc_radius_step(m, cc, rr, dim, 0, len(pip) - 1, vp(pip), vp(pix), vp(cAc),
                                     vp(rAc), np.ascontiguousarray(Ac[0], np.int32),
                                     np.ascontiguousarray(Ac[1], np.int32))
    return rr, cc.reshape(m, dim)


@pytest.mark.parametrize("m,dim", [(2, 3), (3, 3), (17, 2), (40, 3), (300, 4), (1068, 3)])
def test_radius_base_case_device(ctx, oracle, m, dim):
    cA = G.random_coords(m, dim, seed=m)
    r1, c1, dev = ctx.radius_step(cA, dim, True)
    r2, c2 = _oracle_radius(oracle, cA, dim, True)
    assert dev
    assert np.array_equal(r1, r2) and np.array_equal(c1, c2)


@pytest.mark.parametrize("n,draws,seed", [(4096, 40000, 12345), (30000, 240000, 7)])
def test_radius_nonbase_device(ctx, oracle, n, draws, seed):
    A = G.largest_component(G.rmat(n, draws, seed=seed))
    hier = oracle.partition(A, 0.125)
    As = oracle.hierarchy_As(A, hier)
    for l in range(len(hier) - 1):
        m = len(As[l + 1][0]) - 1
        PTc = hier[l + 1]
        cA = G.random_coords(m, 3, seed=l)
        cAc = G.random_coords(PTc[2], 3, seed=l + 10)
        rAc = np.random.RandomState(l).uniform(0.1, 1.0, PTc[2])
        r2, c2 = _oracle_radius(oracle, cA, 3, False, PTc, cAc, rAc, As[l + 1])
        for rep in range(4):  # pops race inside a round: repeat to expose order bugs
            r1, c1, dev = ctx.radius_step(cA, 3, False, PTc=PTc, coords_Ac=cAc, r_Ac=rAc,
                                          Ac=As[l + 1])
            assert dev
            assert np.array_equal(r1, r2) and np.array_equal(c1, c2), (l, rep)


def _one_group(A, cA, oracle, ctx):
    m = len(A[0]) - 1
    PTc = (np.array([0, m], np.int32), np.arange(m, dtype=np.int32))
    cAc = np.array([[0.1, -0.2, 0.3]])
    rAc = np.array([0.7])
    r1, c1, dev = ctx.radius_step(cA, 3, False, PTc=PTc, coords_Ac=cAc, r_Ac=rAc, Ac=A)
    r2, c2 = _oracle_radius(oracle, cA, 3, False, PTc, cAc, rAc, A)
    return r1, c1, dev, r2, c2


@pytest.mark.parametrize("shape", ["star", "path", "grid", "star_upper", "grid_upper"])
def test_radius_group_shapes(ctx, oracle, shape):
    """*_upper: A_c stores only its upper triangle (the reference accepts it,
    src/embed.cpp:697-704): one event per stored entry, nnz events in all."""
    import scipy.sparse as sp
    m = 2000
    upper = shape.endswith("_upper")
    shape = shape.replace("_upper", "")
    if shape == "star":
        e = [(0, j) for j in range(1, m)]
    elif shape == "path":
        e = [(j, j + 1) for j in range(m - 1)]
    else:
        e = [(j, j + 1) for j in range(m - 1) if (j + 1) % 40] + [(j, j + 40) for j in range(m - 40)]
    r = [a for a, b in e] + ([] if upper else [b for a, b in e])
    c = [b for a, b in e] + ([] if upper else [a for a, b in e])
    M = sp.csr_matrix((np.ones(len(r)), (r, c)), shape=(m, m))
    M.sort_indices()
    A = (M.indptr.astype(np.int32), M.indices.astype(np.int32), M.data)
    rs = np.random.RandomState(3)
    cA = np.cumsum(rs.uniform(0.1, 1.0, (m, 3)), axis=0) if shape == "path" else \
        rs.uniform(-1, 1, (m, 3))
    r1, c1, dev, r2, c2 = _one_group(A, cA, oracle, ctx)
    assert dev
    assert np.array_equal(r1, r2) and np.array_equal(c1, c2)


def test_radius_zero_distance_falls_back(ctx, oracle):
    A = G.largest_component(G.rmat(500, 3000, seed=2))
    m = len(A[0]) - 1
    cA = G.random_coords(m, 3, seed=1)
    j = A[1][A[0][0]]  # vertex 0 and a neighbour coincide
    cA[j] = cA[0]
    r1, c1, dev, r2, c2 = _one_group(A, cA, oracle, ctx)
    assert not dev
    assert np.array_equal(r1, r2) and np.array_equal(c1, c2)
