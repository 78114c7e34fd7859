"""libge.so on the CPU: the C ABI loads and exports every symbol include/ge.h
declares, and the host-resident algorithms (partition hierarchy, radius step,
modularity, RNG stream, synthetic inputs) match the oracle bit for bit.
No device calls are made here.
"""
import ctypes

import numpy as np
import pytest

import ge_amd as ge
import graphs as G


def test_library_exports_every_declared_symbol():
    syms = ge.header_symbols()
    assert len(syms) >= 30
    L = ge.lib()
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert b"gfx950" in L.ge_version()


def test_uniform_stream_equals_std(oracle):
    for seed in (0, 1, 12345, 4294967295):
        assert np.array_equal(ge.uniform_stream(seed, 5000), oracle.uniform_stream(seed, 5000))


def test_rmat_generator_matches_definition():
    A = ge.rmat_csr(5000, 40000, seed=3)
    B = G.rmat(5000, 40000, seed=3)
    for a, b in zip(A, B):
        assert np.array_equal(a, b)
    ip, ix, _ = A  # symmetric, sorted, no self loops
    rows = np.repeat(np.arange(5000), np.diff(ip))
    assert not np.any(rows == ix)
    key = set(zip(rows.tolist(), ix.tolist()))
    assert all((c, r) in key for r, c in list(key)[:2000])


def test_largest_component_matches_definition():
    A = ge.rmat_csr(3000, 9000, seed=5)
    for a, b in zip(ge.largest_component(A), G.largest_component(A)):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("n,draws,cf", [(2000, 16000, 0.125), (4096, 40000, 0.125),
                                        (1500, 9000, 0.3)])
def test_partition_bitexact(oracle, n, draws, cf):
    A = G.largest_component(G.rmat(n, draws, seed=n))
    hg = ge.partition(A, cf)
    ho = oracle.partition(A, cf)
    assert len(hg) == len(ho)
    for a, b in zip(hg, ho):
        assert a[2:] == b[2:]
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_partition_er_c1(oracle, golden):
    g = golden("embed_c1_er1000_d2")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    hg = ge.partition(A, 0.1)
    assert len(hg) == int(g["levels"])
    for l, PT in enumerate(hg):
        assert np.array_equal(PT[0], g[f"P{l}_ip"]) and np.array_equal(PT[1], g[f"P{l}_ix"])


def test_partition_options(oracle):
    A = G.largest_component(G.rmat(1200, 8000, seed=77))
    for kw in (dict(positive_merging=False), dict(matching_iterations=1),
               dict(stall=0.99)):
        hg = ge.partition(A, 0.2, **kw)
        ho = oracle.partition(A, 0.2, positive_merging=kw.get("positive_merging", True),
                              stall=kw.get("stall", 1.0),
                              matching=kw.get("matching_iterations", 2))
        assert len(hg) == len(ho)
        for a, b in zip(hg, ho):
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_partition_rejects_merge_leaves():
    A = G.erdos_renyi(30, 0.2)
    with pytest.raises(ge.GeError):
        ge.partition(A, 0.1, merge_leaves=True)


def test_interpolation_matrix():
    ip, ix, dx = ge.interpolation_matrix(6, [[0, 3], [1], [2, 4, 5]])
    assert list(ip) == [0, 2, 3, 6] and list(ix) == [0, 3, 1, 2, 4, 5]
    assert np.all(dx == 1.0)
    with pytest.raises(ge.GeError):  # sizes must sum to numCols (partitioner.cpp:63)
        ge.interpolation_matrix(7, [[0, 3], [1]])


def test_modularity(oracle):
    A = G.largest_component(G.rmat(1000, 6000, seed=1))
    PT = oracle.partition(A, 0.125)[0]
    vA = ge.vertex_of(PT)
    assert ge.modularity(A, vA, PT[2]) == oracle.modularity(A, vA, PT[2])


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


@pytest.mark.parametrize("m", [2, 3, 17, 40])
def test_radius_base_case(oracle, m):
    cA = G.random_coords(m, 3, seed=m)
    r1, c1 = ge.radius_step(cA, 3, True)
    r2, c2 = _oracle_radius(oracle, cA, 3, True)
    assert np.array_equal(r1, r2) and np.array_equal(c1, c2)
    assert np.all(r1 > 0)


def test_radius_nonbase(oracle):
    A = G.largest_component(G.rmat(4096, 40000, seed=12345))
    hier = oracle.partition(A, 0.125)
    As = oracle.hierarchy_As(A, hier)
    for l in range(len(hier) - 1):
        m = len(As[l + 1][0]) - 1
        PTc = hier[l + 1]
        cA = G.random_coords(m, 3, seed=l)
        cAc = G.random_coords(PTc[2], 3, seed=l + 10)
        rAc = np.random.RandomState(l).uniform(0.1, 1.0, PTc[2])
        r1, c1 = ge.radius_step(cA, 3, False, PTc=PTc, coords_Ac=cAc, r_Ac=rAc, Ac=As[l + 1])
        r2, c2 = _oracle_radius(oracle, cA, 3, False, PTc, cAc, rAc, As[l + 1])
        assert np.array_equal(r1, r2) and np.array_equal(c1, c2)


def test_device_entry_points_fail_loudly_without_gpu():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a device is present")
    except ImportError:
        pass
    with pytest.raises(ge.GeError):
        ge.Context(0)


def test_plan_close_reports_teardown_errors(monkeypatch):
    """ge_fa_plan_destroy / ge_faml_plan_destroy return GE_ERR_STATE when a sweep
    hand-over wait timed out after the last step (ge_fa.hip sym_check): close()
    raises it, __del__ swallows it.  The library is replaced by a stub whose
    destroy calls fail, so no device is needed."""
    class Stub:
        def __init__(self):
            self.destroyed = []

        def ge_fa_plan_destroy(self, h):
            self.destroyed.append(h)
            return 4

        ge_faml_plan_destroy = ge_fa_plan_destroy

        def ge_last_error(self):
            return b"symmetric hand-over wait timed out"

    stub = Stub()
    monkeypatch.setattr(ge, "_lib", stub)
    for cls in (ge.FaPlan, ge.FamlPlan):
        plan = cls.__new__(cls)
        plan.h = 1234
        with pytest.raises(ge.GeError, match="hand-over"):
            plan.close()
        assert plan.h is None
        plan.close()  # a second close is a no-op
        plan.h = 99
        plan.__del__()  # swallowed
    assert stub.destroyed == [1234, 99, 1234, 99]


@pytest.mark.parametrize("dim,init", [(2, True), (3, True), (4, False), (3, False)])
def test_embed_via_minimization(oracle, dim, init):
    """ge_embed_via_minimization (host C++, directions on OpenMP threads) against
    the oracle's serial restatement of src/embed.cpp:341-559, bit for bit; n > 64
    takes the threaded path."""
    for n in (1, 2, 12, 90):
        if n == 1:
            A = (np.array([0, 0], np.int32), np.zeros(0, np.int32), np.zeros(0))
        elif n == 2:
            A = (np.array([0, 1, 2], np.int32), np.array([1, 0], np.int32), np.ones(2))
        else:
            A = G.largest_component(G.rmat(n, 4 * n, seed=n))
        m = len(A[0]) - 1
        X0 = None if init else G.random_coords(m, dim, seed=3)
        got = ge.embed_via_minimization(A, dim, coords=X0, iterations=6, seed=17)
        want = oracle.embed_via_minimization(A, dim, coords=X0, iterations=6, seed=17)
        assert np.array_equal(got, want, equal_nan=True), n
