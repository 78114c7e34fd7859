"""The oracle (oracle/ge_oracle.cpp) against the independent pure-Python
restatement (tests/pyref.py) and against the committed golden fixtures.

No reference tests or fixtures exist and the reference
cannot be built here, so these two restatements pin each other; parity with the
reference binary itself is unpinned.
"""
import numpy as np
import pytest

import graphs as G
import pyref as P


def test_mt19937_known_answer():
    # C++11 [rand.predef]: the 10000th output of default-constructed mt19937
    g = P.MT19937(5489)
    for _ in range(9999):
        g()
    assert g() == 4123659995


def test_uniform_stream_matches_libstdcxx(oracle):
    g = P.MT19937(1234)
    want = [P.uniform_m1_p1(g) for _ in range(2000)]
    got = oracle.uniform_stream(1234, 2000)
    assert np.array_equal(np.array(want), got)
    assert got.min() >= -1.0 and got.max() < 1.0


@pytest.mark.parametrize("dim", [1, 2, 3])
def test_force_atlas_supplied_init(oracle, dim):
    A = G.erdos_renyi(50, 0.1, seed=dim)
    X0 = G.random_coords(50, dim, seed=dim)
    py = np.array(P.force_atlas(*G.as_lists(A), dim, coords=X0.tolist(), iterations=12))
    assert np.array_equal(py, oracle.force_atlas(A, dim, coords=X0, iterations=12))


def test_force_atlas_random_init(oracle):
    A = G.largest_component(G.rmat(120, 500, seed=2))
    py = np.array(P.force_atlas(*G.as_lists(A), 3, iterations=6, seed=99))
    assert np.array_equal(py, oracle.force_atlas(A, 3, iterations=6, seed=99))


def test_force_atlas_thread_count_invariant(oracle):
    A = G.erdos_renyi(200, 0.05, seed=1)
    X0 = G.random_coords(200, 3)
    a = oracle.force_atlas(A, 3, coords=X0, iterations=20, nthreads=1)
    b = oracle.force_atlas(A, 3, coords=X0, iterations=20, nthreads=8)
    assert np.array_equal(a, b)


def test_force_atlas_weighted_and_selfloops(oracle):
    # weights other than 1 and a self-loop (contributes +0, include/forceatlas.hpp:169)
    A = G.erdos_renyi(40, 0.15, seed=4)
    ip, ix, dx = (np.array(a) for a in A)
    dx = np.random.RandomState(0).uniform(0.5, 3.0, len(dx))
    rows, cols = [], []
    for i in range(40):
        seg = list(ix[ip[i]:ip[i + 1]])
        w = list(dx[ip[i]:ip[i + 1]])
        if i % 7 == 0:
            seg.append(i)
            w.append(2.0)
        rows.append(sorted(zip(seg, w)))
    nip = np.cumsum([0] + [len(r) for r in rows]).astype(np.int32)
    nix = np.array([c for r in rows for c, _ in r], np.int32)
    ndx = np.array([w for r in rows for _, w in r], np.float64)
    X0 = G.random_coords(40, 2, seed=9)
    py = np.array(P.force_atlas(list(nip), list(nix), list(ndx), 2, coords=X0.tolist(),
                                iterations=8))
    assert np.array_equal(py, oracle.force_atlas((nip, nix, ndx), 2, coords=X0, iterations=8))


def test_force_atlas_ml(oracle):
    A = G.largest_component(G.rmat(600, 3000, seed=5))
    hier = oracle.partition(A, 0.125)
    PT = hier[0]
    vA = oracle.vertex_of(PT)
    cA = G.random_coords(PT[2], 3, seed=11)
    rA = np.random.RandomState(3).uniform(0.1, 0.5, PT[2])
    py = np.array(P.force_atlas_ml(*G.as_lists(A), list(PT[0]), list(PT[1]), list(vA),
                                   cA.tolist(), rA.tolist(), 3, 8, 77))
    o1 = oracle.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=8, seed=77, nthreads=1)
    o8 = oracle.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=8, seed=77, nthreads=8)
    assert np.array_equal(py, o1)
    assert np.array_equal(o1, o8)


@pytest.mark.parametrize("cf", [0.3, 0.125])
def test_partition(oracle, cf):
    A = G.largest_component(G.rmat(900, 5000, seed=6))
    hp = P.partition(*G.as_lists(A), cf)
    ho = oracle.partition(A, cf)
    assert len(hp) == len(ho) >= 1
    for a, b in zip(hp, ho):
        assert a[2:] == b[2:]
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("case", ["rmat", "hubs", "er", "weights", "nopos", "stall", "match3"])
def test_partition_flat_equals_map(oracle, case):
    """orc_partition_flat (unordered entry lists, used for the C4 digest) against
    orc_partition (the reference's std::map): identical hierarchies with every
    option, fractional weights (several entries of equal eta), hub lists past the
    index threshold."""
    kw = {}
    if case == "er":
        A = G.erdos_renyi(1500, 0.008, seed=3)
    elif case == "hubs":
        A = G.with_hubs(G.largest_component(G.rmat(3000, 20000, seed=8)), [(5, 1500), (9, 800)])
    else:
        A = G.largest_component(G.rmat(4000, 30000, seed=10))
    if case == "weights":  # symmetric weights from a few values: ties in eta
        ip, ix, dx = A
        rows = np.repeat(np.arange(len(ip) - 1), np.diff(ip))
        w = 1.0 + ((np.minimum(rows, ix) * 7 + np.maximum(rows, ix) * 13) % 3) * 0.5
        A = (ip, ix, w)
    if case == "nopos":
        kw = dict(positive_merging=False)
    if case == "stall":
        kw = dict(stall=0.97)
    if case == "match3":
        kw = dict(matching=3)
    for cf in (0.125, 0.4):
        hm = oracle.partition(A, cf, **kw)
        hf = oracle.partition(A, cf, flat=True, **kw)
        assert len(hm) == len(hf) >= 1
        for a, b in zip(hm, hf):
            assert a[2:] == b[2:]
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_partition_shapes_chain(oracle):
    A = G.largest_component(G.rmat(2000, 14000, seed=7))
    hier = oracle.partition(A, 0.125)
    n = len(A[0]) - 1
    for PT in hier:  # cols of level l == rows of level l-1, one entry per column
        assert PT[3] == n and PT[0][-1] == n
        assert np.array_equal(np.sort(PT[1]), np.arange(n))
        n = PT[2]


def test_ptap_dense(oracle):
    A = G.largest_component(G.rmat(300, 1500, seed=9))
    ip, ix, dx = A
    n = len(ip) - 1
    hier = oracle.partition(A, 0.3)
    PT = hier[0]
    Pm = np.zeros((PT[2], n))
    for a in range(PT[2]):
        Pm[a, PT[1][PT[0][a]:PT[0][a + 1]]] = 1.0
    Ad = np.zeros((n, n))
    for i in range(n):
        Ad[i, ix[ip[i]:ip[i + 1]]] = dx[ip[i]:ip[i + 1]]
    C = oracle.ptap(A, PT)
    Cd = np.zeros((PT[2], PT[2]))
    for a in range(PT[2]):
        assert np.all(np.diff(C[1][C[0][a]:C[0][a + 1]]) > 0)  # rows sorted ascending
        Cd[a, C[1][C[0][a]:C[0][a + 1]]] = C[2][C[0][a]:C[0][a + 1]]
    assert np.array_equal(Cd, Pm @ Ad @ Pm.T)


def test_golden_fixtures_reproduce(oracle, golden):
    g = golden("fa_er300_d3")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    for it in (1, 10, 100):
        assert np.array_equal(oracle.force_atlas(A, 3, coords=g["x0"], iterations=it),
                              g[f"x_it{it}"])
    g = golden("fa_rmat_d2_seeded")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    assert np.array_equal(oracle.force_atlas(A, 2, iterations=20, seed=int(g["seed"])),
                          g["x_it20"])
    g = golden("partition_rmat4096")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    hier = oracle.partition(A, 0.125)
    assert len(hier) == int(g["levels"])
    for l, PT in enumerate(hier):
        assert np.array_equal(PT[0], g[f"P{l}_ip"]) and np.array_equal(PT[1], g[f"P{l}_ix"])
    g = golden("faml_rmat4096_l0")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    X = oracle.force_atlas_ml(A, (g["P_ip"], g["P_ix"]), g["vA"], g["cA"], g["rA"], 3,
                              iterations=100, seed=int(g["seed"]))
    assert np.array_equal(X, g["x_it100"])


def test_golden_c1_embed(oracle, golden):
    g = golden("embed_c1_er1000_d2")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    hier = oracle.partition(A, 0.1)
    assert [h[2] for h in hier] == [int(g[f"P{l}_shape"][0]) for l in range(int(g["levels"]))]
    As = oracle.hierarchy_As(A, hier)
    X = oracle.embed(As, hier, 2, seed=int(g["seed"]))
    assert np.array_equal(X, g["coords"])
    assert np.isfinite(X).all()  # examples/embedder.cpp:224-228
