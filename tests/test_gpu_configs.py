"""Device parity at the BASELINE configs' own sizes (configs[1] to [4]) plus the
reference options the small-graph suites do not cover.

The dynamics are chaotic and every kernel is strict fp64 in the reference's op
order, so the bar is bit-exact (np.array_equal) against the oracle
(oracle/ge_oracle.cpp) evaluated on a SAMPLE of rows / aggregates: the oracle is
the reference's serial loop, and a whole configs[1] iteration (1e12 pair terms)
or configs[2] level (4e11 per 100 iterations) is out of reach for it in a test.

* configs[1] (C2): one full forceAtlas iteration of the 1M-id R-MAT on the device;
  the oracle steps ~300 rows -- the first / last / middle rows, the 32 heaviest
  rows (segment-split hub rows, include/forceatlas.hpp:169-203) and random rows.
* configs[2] (C3): the level-0 forceAtlasMultilevel call (100 iterations) of the
  1M-id R-MAT LCC, hierarchy from the device partition; the oracle evaluates the
  aggregates around the resident / streamed split, the four smallest above 2000
  members (streamed queue path) and 150 random small ones, with the same draw
  stream (:340-360, single-thread order).
* configs[4] (C5): the attraction / gravity / update pass (ge_fa_plan_attract) of
  the 100M-id / 800M-draw R-MAT (nnz 1.41e9, hub rows of 652 499 entries) on
  supplied repulsion sums; the oracle steps ~200 rows incl. the 24 largest hubs.
* nohubs (plain division: bit-exact), linlog / delta != 1 (device log / pow: within
  1e-12 relative after one iteration), modularity on the device vs the oracle.
"""
import numpy as np
import pytest
import torch

import ge_amd as ge
import graphs as G

pytestmark = pytest.mark.gpu


def _rows_sample(n, deg, rng, heavy=32, rand=64, edge=64):
    rows = set(range(edge)) | set(range(n - edge, n)) | set(range(n // 2, n // 2 + edge))
    rows |= set(np.argpartition(-deg, heavy)[:heavy].tolist())  # the heaviest rows
    rows |= set(rng.integers(0, n, rand).tolist())
    return np.array(sorted(rows), dtype=np.int64)


def _progress(t0, what):
    import sys
    import time
    print(f"[{time.perf_counter() - t0:6.1f}s] {what}", file=sys.stderr, flush=True)


def test_c2_full_size_iteration_sampled_rows(ctx, oracle):
    A = ge.rmat_csr(1_000_000, 8_000_000, seed=12345)
    n = len(A[0]) - 1
    X0 = ge.uniform_stream(12345, n * 3).reshape(n, 3)
    got = ctx.force_atlas(A, 3, coords=X0, iterations=1)
    deg = oracle.degrees(A)
    rows = _rows_sample(n, np.diff(A[0]), np.random.default_rng(1))
    want = X0.copy()
    # one row per call (the oracle's fa_step_rows works on [rb, re)); no thread-count
    # override: omp_set_num_threads would also bind libge's later OpenMP regions
    for r in rows:
        fprev = np.zeros((1, 3))
        oracle.fa_step_rows(A, X0, deg, int(r), int(r) + 1, fprev, want)
    assert np.array_equal(got[rows], want[rows])
    assert np.isfinite(got).all()


def test_c3_level0_sampled_aggregates(ctx, oracle):
    L = ge.largest_component(ge.rmat_csr(1_000_000, 8_000_000, seed=12345))
    PT = ctx.partition(L, 0.125)[0]
    m = PT[2]
    vA = ge.vertex_of(PT)
    cA = ge.uniform_stream(7, m * 3).reshape(m, 3)
    rA = 0.01 + 0.19 * (ge.uniform_stream(8, m) + 1.0) / 2.0
    got = ctx.force_atlas_ml(L, PT, vA, cA, rA, 3, iterations=100, seed=5)
    sizes = np.diff(PT[0])
    order = np.argsort(sizes, kind="stable")
    big = [a for a in order if sizes[a] > 2000][:4]
    split = [a for a in order if 200 <= sizes[a] <= 2000][-6:]  # around the resident cap
    small = np.random.default_rng(2).choice(np.nonzero(sizes <= 200)[0], 150, replace=False)
    aggs = np.array(sorted(set(big) | set(split) | set(small.tolist())), dtype=np.int32)
    want = oracle.force_atlas_ml_aggs(L, PT, vA, cA, rA, 3, aggs, iterations=100, seed=5)
    rows = np.concatenate([PT[1][PT[0][a]:PT[0][a + 1]] for a in aggs])
    assert len(big) == 4 and sizes[aggs].max() > 2000
    assert np.array_equal(got[rows], want[rows])
    assert np.isfinite(got).all()


def test_c4_level0_sampled_aggregates(ctx, oracle, heartbeat):
    """configs[3] (C4, the headline): the 10M-id R-MAT LCC (n = 4.39M), device
    partition, level-0 forceAtlasMultilevel (2 iterations: the symmetric streamed
    kernel with its sweep hand-overs at full size) against the oracle on the largest
    aggregate (41 930 members), aggregates around the streamed / resident split and
    random small ones."""
    import time
    t0 = time.perf_counter()
    L = ge.largest_component(ge.rmat_csr(10_000_000, 80_000_000, seed=12345))
    _progress(t0, f"C4 LCC n={len(L[0]) - 1}")
    PT = ctx.partition(L, 0.125)[0]
    _progress(t0, "C4 device partition")
    m = PT[2]
    vA = ge.vertex_of(PT)
    cA = ge.uniform_stream(7, m * 3).reshape(m, 3)
    rA = 0.01 + 0.19 * (ge.uniform_stream(8, m) + 1.0) / 2.0
    got = ctx.force_atlas_ml(L, PT, vA, cA, rA, 3, iterations=2, seed=5)
    _progress(t0, "C4 device level done")
    sizes = np.diff(PT[0])
    order = np.argsort(sizes, kind="stable")
    big = [int(order[-1])] + [a for a in order if 2000 < sizes[a] <= 4000][:3]
    split = [a for a in order if 200 <= sizes[a] <= 2000][-4:]
    small = np.random.default_rng(4).choice(np.nonzero(sizes <= 200)[0], 100, replace=False)
    aggs = np.array(sorted(set(big) | set(split) | set(small.tolist())), dtype=np.int32)
    with heartbeat("C4 oracle aggregates"):
        want = oracle.force_atlas_ml_aggs(L, PT, vA, cA, rA, 3, aggs, iterations=2, seed=5)
    _progress(t0, "C4 oracle aggregates done")
    rows = np.concatenate([PT[1][PT[0][a]:PT[0][a + 1]] for a in aggs])
    assert sizes[aggs].max() > 40000
    assert np.array_equal(got[rows], want[rows])
    assert np.isfinite(got).all()


def test_c4_level0_oracle_at_embed_horizon(ctx, golden, monkeypatch, heartbeat):
    """configs[3] (C4) level 0 at the embed's own horizon, 100 iterations
    (src/embed.cpp:793), against the oracle's 100 iterations
    (tests/golden/make_c4_level0_100.py; 1 301 s on 8 threads) on the largest aggregate
    (41 930 members: the longest sweep chain), the two smallest streamed and the two
    largest LDS-resident aggregates (the size-class boundary) and 100 random small
    ones.  The shipped schedule (symmetric sweeps at N = 1) and every streamed
    aggregate as ordered row blocks (the multi-GPU shares' schedule,
    GE_FAML_SYM_CHAIN=1e9) must both equal the oracle bit for bit."""
    import hashlib
    import time
    t0 = time.perf_counter()
    g = golden("faml_c4_level0_100it")
    L = ge.largest_component(ge.rmat_csr(10_000_000, 80_000_000, seed=12345))
    PT = ctx.partition(L, 0.125)[0]
    _progress(t0, "C4 device partition")
    lvl0 = hashlib.sha256(np.ascontiguousarray(PT[0], np.int32).tobytes() +
                          np.ascontiguousarray(PT[1], np.int32).tobytes()).hexdigest()
    assert lvl0 == str(g["level0_sha256"])
    aggs = g["aggs"]
    h = hashlib.sha256()
    for a in aggs:
        h.update(np.ascontiguousarray(PT[1][PT[0][a]:PT[0][a + 1]], np.int32).tobytes())
    assert h.hexdigest() == str(g["members_sha256"])
    m = PT[2]
    vA = ge.vertex_of(PT)
    cA = ge.uniform_stream(7, m * 3).reshape(m, 3)
    rA = 0.01 + 0.19 * (ge.uniform_stream(8, m) + 1.0) / 2.0
    rows = g["rows"].astype(np.int64)
    assert np.diff(PT[0])[aggs].max() == 41930
    for name, env in (("shipped", {}), ("row_blocks", {"GE_FAML_SYM_CHAIN": "1e9"})):
        for k in ("GE_FAML_SYM_CHAIN",):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        with heartbeat(f"C4 level 0, 100 iterations, {name}"):
            got = ctx.force_atlas_ml(L, PT, vA, cA, rA, 3, iterations=int(g["iterations"]),
                                     seed=int(g["seed"]))
        _progress(t0, f"C4 {name} done")
        assert np.isfinite(got).all()
        assert np.array_equal(got[rows], g["x"]), name


def test_c4_level0_schedules_agree_at_embed_horizon(ctx, monkeypatch, heartbeat):
    """C4 level 0 over the embed's 100 iterations (src/embed.cpp:793): the streamed
    aggregates (98 at C4, up to 41 930 members) as symmetric sweeps (the default), as
    ordered row blocks (GE_FAML_SYM_CHAIN=1e9) and through the ordered-pair kernel
    (GE_FAML_SYM=0) give the same bits.  Each schedule is pinned to the oracle on
    small levels (test_gpu_parity.py) and at C4 for 2 iterations above; the oracle
    would need hours for 100 iterations of these aggregates, so the long horizon is
    checked as agreement of three independent schedules (a hand-over or queue-order
    fault shows as a difference)."""
    import time
    t0 = time.perf_counter()
    L = ge.largest_component(ge.rmat_csr(10_000_000, 80_000_000, seed=12345))
    PT = ctx.partition(L, 0.125)[0]
    _progress(t0, "C4 device partition")
    m = PT[2]
    vA = ge.vertex_of(PT)
    cA = ge.uniform_stream(7, m * 3).reshape(m, 3)
    rA = 0.01 + 0.19 * (ge.uniform_stream(8, m) + 1.0) / 2.0
    runs = {}
    for name, env in (("sweeps", {}), ("row_blocks", {"GE_FAML_SYM_CHAIN": "1e9"}),
                      ("ordered_pairs", {"GE_FAML_SYM": "0"})):
        for k in ("GE_FAML_SYM_CHAIN", "GE_FAML_SYM"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        with heartbeat(f"C4 level 0, 100 iterations, {name}"):
            runs[name] = ctx.force_atlas_ml(L, PT, vA, cA, rA, 3, iterations=100, seed=5)
        _progress(t0, f"C4 {name} done")
    assert np.isfinite(runs["sweeps"]).all()
    assert np.array_equal(runs["sweeps"], runs["row_blocks"])
    assert np.array_equal(runs["sweeps"], runs["ordered_pairs"])


def test_c4_embed_end_to_end_schedules_agree(ctx, monkeypatch, heartbeat):
    """The whole C4 embed (examples/embed.cpp: 4 levels of the device partition,
    P^T A P, the coarsest level's 1e5 iterations, radius steps, 100 multilevel
    iterations per level) with the shipped kernels -- symmetric sweeps, packed
    coarsest rows -- and with the independent ones -- the ordered-pair multilevel
    kernel (GE_FAML_SYM=0), one wave per coarsest row (GE_FA_PACKED=0): the same
    bits end to end (bench.py checks only finiteness)."""
    import time
    t0 = time.perf_counter()
    L = ge.largest_component(ge.rmat_csr(10_000_000, 80_000_000, seed=12345))
    hier = ctx.partition(L, 0.125)[:4]
    As = [L]
    for PT in hier:
        As.append(ctx.ptap(As[-1], PT))
    _progress(t0, "C4 hierarchy and P^T A P")
    runs = {}
    for name, env in (("shipped", {}), ("independent", {"GE_FAML_SYM": "0", "GE_FA_PACKED": "0"})):
        for k in ("GE_FAML_SYM", "GE_FA_PACKED"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        with heartbeat(f"C4 embed, {name} kernels"):
            runs[name] = ctx.embed(As, hier, 3, seed=12345)
        _progress(t0, f"C4 embed {name} done")
    assert np.isfinite(runs["shipped"]).all()
    assert np.array_equal(runs["shipped"], runs["independent"])


def _coarse_rows_numpy(L, PT, vA, rows):
    """Rows of P_T A P for the coarse ids `rows`, straight from the definition (entry
    (a, b) = sum of a_ij over i in a, j in b): exact, since the
    R-MAT weights are 1.0."""
    ip, ix, dx = L
    out = {}
    for a in rows:
        mem = PT[1][PT[0][a]:PT[0][a + 1]]
        e = np.concatenate([np.arange(ip[i], ip[i + 1]) for i in mem])
        b, w = np.unique(vA[ix[e]], return_inverse=True)
        out[int(a)] = (b.astype(np.int32), np.bincount(w, weights=dx[e]))
    return out


def test_c5_level0_sampled_aggregates(ctx, oracle, heartbeat):
    """configs[4] (C5) as an embed level: the 100M-id / 800M-draw R-MAT's LCC built
    on the device (examples/embedder.cpp:35-93), partition(A, 0.125) on the device
    (src/partitioner.cpp:1550-1893), P^T A P of level 0 on the device, and the
    level-0 forceAtlasMultilevel call (include/forceatlas.hpp:314-574; 2 iterations,
    symmetric streamed kernel at full size) against the oracle on the largest
    aggregate, the streamed / resident boundary and random small aggregates.  The
    coarse rows of the sampled aggregates are checked against their definition."""
    import os
    import time
    t0 = time.perf_counter()
    L = ctx.rmat_csr(100_000_000, 800_000_000, seed=12345, lcc=True)
    n, nnz = len(L[0]) - 1, len(L[1])
    _progress(t0, f"C5 LCC n={n} nnz={nnz} (device)")
    with heartbeat("C5 device partition"):
        hier = ctx.partition(L, 0.125)
    _progress(t0, f"C5 device partition levels {[h[2] for h in hier]}")
    PT = hier[0]
    m = PT[2]
    assert PT[3] == n and len(PT[1]) == n
    assert np.array_equal(np.sort(PT[1]), np.arange(n, dtype=np.int32))
    vA = ge.vertex_of(PT)
    C = ctx.ptap(L, PT)
    _progress(t0, f"C5 device P^T A P nnz={len(C[1])}")
    assert len(C[0]) == m + 1 and C[2].sum() == L[2].sum()
    sizes = np.diff(PT[0])
    order = np.argsort(sizes, kind="stable")
    big = [int(order[-1])] + [int(a) for a in order if 2000 < sizes[a] <= 4000][:3]
    split = [int(a) for a in order if 200 <= sizes[a] <= 2000][-4:]
    small = np.random.default_rng(6).choice(np.nonzero(sizes <= 200)[0], 100, replace=False)
    aggs = np.array(sorted(set(big) | set(split) | set(small.tolist())), dtype=np.int32)
    for a, (b, w) in _coarse_rows_numpy(L, PT, vA, aggs).items():
        assert np.array_equal(C[1][C[0][a]:C[0][a + 1]], b)
        assert np.array_equal(C[2][C[0][a]:C[0][a + 1]], w)
    del C
    cA = ge.uniform_stream(7, m * 3).reshape(m, 3)
    rA = 0.01 + 0.19 * (ge.uniform_stream(8, m) + 1.0) / 2.0
    with heartbeat("C5 level 0"):
        got = ctx.force_atlas_ml(L, PT, vA, cA, rA, 3, iterations=2, seed=5)
    _progress(t0, f"C5 device level done (largest aggregate {sizes.max()})")
    with heartbeat("C5 oracle aggregates"):
        want = oracle.force_atlas_ml_aggs(L, PT, vA, cA, rA, 3, aggs, iterations=2, seed=5)
    _progress(t0, "C5 oracle aggregates done")
    rows = np.concatenate([PT[1][PT[0][a]:PT[0][a + 1]] for a in aggs])
    assert sizes[aggs].max() == sizes.max()
    assert np.array_equal(got[rows], want[rows])
    assert np.isfinite(got).all()


def test_c5_attraction_pass_sampled_rows(oracle, heartbeat):
    import time
    t0 = time.perf_counter()
    with heartbeat("C5 host R-MAT"):
        A = ge.rmat_csr(100_000_000, 800_000_000, seed=12345)
    _progress(t0, "C5 graph generated")
    n, nnz = len(A[0]) - 1, int(A[0][-1])
    dev = torch.device("cuda:0")
    deg_i = np.diff(A[0])
    rng = np.random.default_rng(3)
    rows = _rows_sample(n, deg_i, rng, heavy=24, rand=48, edge=40)
    # inputs defined on the host so the oracle sees the same values
    X = ge.uniform_stream(99, n * 3).reshape(n, 3)
    frep_rows = (ge.uniform_stream(98, len(rows) * 3).reshape(len(rows), 3) *
                 ((deg_i[rows] + 1.0) * 1e6)[:, None])
    ip, ix, dx = (torch.from_numpy(a).to(dev) for a in A)
    x = torch.from_numpy(X).to(dev)
    frep = torch.zeros((n, 3), dtype=torch.float64, device=dev)
    frep[torch.from_numpy(rows).to(dev)] = torch.from_numpy(frep_rows).to(dev)
    y = torch.empty_like(x)
    _progress(t0, "C5 inputs on the device")
    c = ge.Context(0)
    try:
        plan = c.fa_plan(n, nnz, ip.data_ptr(), ix.data_ptr(), dx.data_ptr(), 3, 0, n)
        plan.attract(x.data_ptr(), frep.data_ptr(), y.data_ptr())
        c.sync()
        got = y[torch.from_numpy(rows).to(dev)].cpu().numpy()
        plan.close()
    finally:
        c.close()
    del ip, ix, dx, x, y, frep
    _progress(t0, "C5 device pass done")
    assert deg_i[rows].max() > 600_000  # the hub rows are in the sample
    deg = oracle.degrees(A)
    want = X.copy()
    for r, fr in zip(rows, frep_rows):
        fprev = np.zeros((1, 3))
        oracle.fa_step_rows_frep(A, X, deg, int(r), int(r) + 1, fr[None, :], fprev, want)
    _progress(t0, "C5 oracle rows done")
    assert np.array_equal(got, want[rows])


@pytest.mark.parametrize("n,draws", [(3000, 20000), (30000, 200000)])
def test_nohubs_bitexact(ctx, oracle, n, draws):
    A = G.largest_component(G.rmat(n, draws, seed=n))
    X0 = G.random_coords(len(A[0]) - 1, 3, seed=3)
    got = ctx.force_atlas(A, 3, coords=X0, iterations=3, nohubs=1)
    want = oracle.force_atlas(A, 3, coords=X0, iterations=3, nohubs=1)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("kw", [dict(linlog=1), dict(delta=2.0), dict(delta=0.5, linlog=1)])
def test_linlog_delta_tolerance(ctx, oracle, kw):
    """Device log / pow (ocml) against glibc: 1e-12 relative after one iteration
    (the dynamics amplify last-ulp differences afterwards)."""
    A = G.largest_component(G.rmat(3000, 20000, seed=4))
    X0 = G.random_coords(len(A[0]) - 1, 3, seed=5)
    got = ctx.force_atlas(A, 3, coords=X0, iterations=1, **kw)
    want = oracle.force_atlas(A, 3, coords=X0, iterations=1, **kw)
    assert np.allclose(got, want, rtol=1e-12, atol=0.0)


def test_modularity_device_vs_oracle(ctx, oracle):
    for A, cf in ((G.largest_component(G.rmat(20000, 150000, seed=6)), 0.125),
                  (G.erdos_renyi(1000, 0.01, seed=42), 0.1)):
        hier = oracle.partition(A, cf)
        for Al, PT in zip(oracle.hierarchy_As(A, hier), hier):  # P_T[l] partitions As[l]
            vA = ge.vertex_of(PT)
            assert ctx.modularity(Al, vA, PT[2]) == oracle.modularity(Al, vA, PT[2])
