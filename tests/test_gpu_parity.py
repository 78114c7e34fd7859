"""GPU parity: the HIP path through the C ABI against the oracle and the golden
fixtures.  STRICT mode must be bit-identical (fp64 == fp64, same bits); FAST
mode must stay within the north star's 1e-5 relative bar.
"""
import numpy as np
import pytest

import ge_amd as ge
import graphs as G

pytestmark = pytest.mark.gpu

REL_TOL_FAST = 1e-5  # north star: coordinates within 1e-5 relative


def rel_err(x, ref):
    return float(np.max(np.abs(x - ref)) / np.max(np.abs(ref)))


# --------------------------------------------------------------------------
# exact arithmetic building blocks

def test_shared_reciprocal_division_is_ieee(ctx):
    # 2^30 draws (those whose operands lie in the exact-division domain -- most of
    # them -- are compared): every repulsion term of pair_den against the rcp-based
    # reciprocals and against `/`, bitwise (ge_selftest.hip, ge_pair.hpp pair_den)
    assert ctx.selftest_math(1 << 30, seed=7) == 0


# --------------------------------------------------------------------------
# single-level forceAtlas

@pytest.mark.parametrize("small_max", ["0", "512"])  # grouped multi-block / one workgroup
def test_fa_golden_supplied_init(ctx, golden, monkeypatch, small_max):
    monkeypatch.setenv("GE_SMALL_MAX", small_max)
    g = golden("fa_er300_d3")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    for it in (1, 10, 100):
        X = ctx.force_atlas(A, 3, coords=g["x0"], iterations=it)
        assert np.array_equal(X, g[f"x_it{it}"]), it


def test_fa_golden_random_init(ctx, golden):
    g = golden("fa_rmat_d2_seeded")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    X = ctx.force_atlas(A, 2, iterations=20, seed=int(g["seed"]))
    assert np.array_equal(X, g["x_it20"])


@pytest.mark.parametrize("dim", [1, 2, 3, 4])
def test_fa_small_kernel_dims(ctx, oracle, monkeypatch, dim):
    monkeypatch.setenv("GE_SMALL_MAX", "512")
    A = G.erdos_renyi(97, 0.06, seed=dim)
    X0 = G.random_coords(97, dim, seed=dim)
    want = oracle.force_atlas(A, dim, coords=X0, iterations=30)
    assert np.array_equal(ctx.force_atlas(A, dim, coords=X0, iterations=30), want)


@pytest.mark.parametrize("n,dim", [(1025, 3), (3000, 3), (2500, 2), (1300, 4)])
def test_fa_tiled_kernel_bitexact(ctx, oracle, n, dim):
    A = G.rmat(n, 8 * n, seed=n)  # isolated vertices included (gravity only)
    m = len(A[0]) - 1
    assert m > 1024  # the multi-block (plan) path, not the one-workgroup path
    X0 = G.random_coords(m, dim, seed=1)
    want = oracle.force_atlas(A, dim, coords=X0, iterations=5)
    assert np.array_equal(ctx.force_atlas(A, dim, coords=X0, iterations=5), want)


@pytest.mark.parametrize("tiles", ["0", "1"])
@pytest.mark.parametrize("use_weights", [1, 0])
def test_fa_degree_classes(ctx, oracle, monkeypatch, use_weights, tiles):
    """Rows of every degree class of the attraction kernel (ge_rows.hpp): light,
    wave-per-row (> 32 edges) and block-per-row (> 2048 edges, several chunks);
    with GE_ROWS_TILES=1 the tiles (<= 1024 entries) and block-per-row beyond."""
    monkeypatch.setenv("GE_STREAM_MAX", "0")  # the large-level kernels
    monkeypatch.setenv("GE_ROWS_TILES", tiles)
    A = G.with_hubs(G.rmat(6000, 30000, seed=11), [(5, 4500), (17, 2100), (900, 300)])
    A = (A[0], A[1], np.random.RandomState(2).uniform(0.5, 2.0, len(A[1])))
    deg = np.diff(A[0])
    assert deg.max() > 4096 and ((deg > 32) & (deg <= 2048)).any()
    X0 = G.random_coords(len(deg), 3, seed=4)
    want = oracle.force_atlas(A, 3, coords=X0, iterations=4, use_weights=use_weights)
    got = ctx.force_atlas(A, 3, coords=X0, iterations=4, use_weights=use_weights)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("segments", ["1", "0"])
@pytest.mark.parametrize("dim", [1, 2, 3, 4])
def test_fa_row_tiles(ctx, oracle, monkeypatch, dim, segments):
    """Tiled CSR rows: rows at and around the tile capacity (tile vs heavy),
    tiles closed by the row limit and by the entry limit, isolated rows, every
    dimension; heavy rows as binade-sum segments or whole rows (GE_ROWS_SEGMENTS)."""
    monkeypatch.setenv("GE_STREAM_MAX", "0")  # the large-level kernels
    monkeypatch.setenv("GE_ROWS_TILES", "1")
    monkeypatch.setenv("GE_ROWS_SEGMENTS", segments)
    A = G.with_degrees(G.rmat(5000, 20000, seed=dim), {7: 1023, 8: 1024, 9: 1025, 300: 700,
                                                       301: 400, 4000: 1500}, seed=dim)
    deg = np.diff(A[0])
    assert list(deg[[7, 8, 9, 300]]) == [1023, 1024, 1025, 700] and (deg == 0).any()
    X0 = G.random_coords(len(deg), dim, seed=dim)
    want = oracle.force_atlas(A, dim, coords=X0, iterations=3)
    assert np.array_equal(ctx.force_atlas(A, dim, coords=X0, iterations=3), want)


@pytest.mark.parametrize("scale", [1.0, 1e9, 1e-300])
def test_fa_heavy_segments_binade_and_fallback(ctx, oracle, monkeypatch, scale):
    """Heavy rows split into segments whose terms are summed as integers in the
    binade of the repulsion sum.  Edge weights of 1e9 make the terms too large
    for the binade (|t/ulp| >= 2^36) and 1e-300 pushes the weighted degrees (and
    so the repulsion sums) towards the subnormal range: both fall back to the
    serial in-order sum.  Bit-exact either way."""
    monkeypatch.setenv("GE_STREAM_MAX", "0")  # the large-level kernels
    monkeypatch.setenv("GE_ROWS_TILES", "1")
    A = G.with_degrees(G.rmat(7000, 28000, seed=4), {3: 5000, 11: 2600, 12: 513}, seed=5)
    A = (A[0], A[1], A[2] * scale)
    X0 = G.random_coords(7000, 3, seed=9)
    for it in (1, 3):
        want = oracle.force_atlas(A, 3, coords=X0, iterations=it)
        got = ctx.force_atlas(A, 3, coords=X0, iterations=it)
        assert np.array_equal(got, want), it


def test_fa_row_tiles_graph_replay(ctx, oracle, monkeypatch):
    """Tiles + heavy rows on the side stream inside a captured graph (>= 128
    iterations replay 32-iteration graphs with the fork/join events)."""
    monkeypatch.setenv("GE_STREAM_MAX", "0")  # the large-level kernels
    monkeypatch.setenv("GE_ROWS_TILES", "1")
    A = G.with_degrees(G.rmat(3300, 12000, seed=21), {5: 1500, 6: 900}, seed=2)
    X0 = G.random_coords(3300, 2, seed=6)
    want = oracle.force_atlas(A, 2, coords=X0, iterations=130)
    assert np.array_equal(ctx.force_atlas(A, 2, coords=X0, iterations=130), want)


@pytest.mark.parametrize("R", ["1", "2", "4", "8"])
def test_fa_repulsion_row_slots(ctx, oracle, monkeypatch, R):
    """fa_repulse_strict with R row slots x 8/R partners in flight per lane
    (row shards of N GPUs pick small R), ragged tiles and slot counts."""
    monkeypatch.setenv("GE_STREAM_MAX", "0")  # the large-level kernels
    monkeypatch.setenv("GE_FA_SYM", "0")  # the ordered-pair kernel (row shards use it)
    monkeypatch.setenv("GE_REP_R", R)
    A = G.rmat(9000, 60000, seed=3)
    n = len(A[0]) - 1
    X0 = G.random_coords(n, 3, seed=8)
    want = oracle.force_atlas(A, 3, coords=X0, iterations=3)
    assert np.array_equal(ctx.force_atlas(A, 3, coords=X0, iterations=3), want)


@pytest.mark.parametrize("R", ["1", "2", "4", "8"])
def test_fa_repulsion_full_row_slots(ctx, oracle, monkeypatch, R):
    """Blocks that own thousands of rows, as at C2 (1M rows over 256 CUs): every
    row slot of a wave is filled (the branch-free path with the partner's
    record read once for all R rows), plus the ragged last chunk."""
    monkeypatch.setenv("GE_STREAM_MAX", "0")
    monkeypatch.setenv("GE_FA_SYM", "0")  # the ordered-pair kernel (row shards use it)
    monkeypatch.setenv("GE_REP_R", R)
    monkeypatch.setenv("GE_REP_BLOCKS", "2")  # 4544 rows per block
    A = G.rmat(9000, 60000, seed=5)
    n = len(A[0]) - 1
    X0 = G.random_coords(n, 3, seed=9)
    want = oracle.force_atlas(A, 3, coords=X0, iterations=3)
    assert np.array_equal(ctx.force_atlas(A, 3, coords=X0, iterations=3), want)


@pytest.mark.parametrize("n,dim,repel", [(9000, 3, 1.0), (5000, 1, 1.0), (4097, 2, 1.0),
                                          (3000, 4, 1.0), (6500, 3, 1.7), (64, 3, 1.0),
                                          (65, 2, 1.0), (200, 3, 1e21)])
def test_fa_symmetric_repulsion(ctx, oracle, monkeypatch, n, dim, repel):
    """Single-level forceAtlas with the symmetric sweeps (ge_sym.hpp): the level as
    one aggregate of ceil(n / 64) row tiles, each unordered pair evaluated once,
    column sums handed from sweep to sweep; ragged last tile, one and two tiles,
    every dimension, repel != 1 and a repel large enough (1e21) to leave the
    shared-reciprocal domain (the `/` forms)."""
    monkeypatch.setenv("GE_STREAM_MAX", "0")
    monkeypatch.setenv("GE_FA_SYM", "1")
    A = G.rmat(n, 6 * n, seed=n + dim)
    m = len(A[0]) - 1
    X0 = G.random_coords(m, dim, seed=dim)
    want = oracle.force_atlas(A, dim, coords=X0, iterations=3, repel=repel)
    assert np.array_equal(ctx.force_atlas(A, dim, coords=X0, iterations=3, repel=repel), want)


def test_fa_symmetric_repulsion_domain_and_ties(ctx, oracle, monkeypatch):
    """Symmetric sweeps with a coordinate outside the exact-division domain (its
    tiles take the `/` forms), coincident points (distance clamped to eps) and
    isolated vertices, over enough iterations to replay a captured graph."""
    monkeypatch.setenv("GE_STREAM_MAX", "0")
    monkeypatch.setenv("GE_FA_SYM", "1")
    A = G.rmat(3000, 12000, seed=44)
    X0 = G.random_coords(3000, 3, seed=8)
    X0[1500, 1] = 1e-70
    X0[10] = X0[11]
    want = oracle.force_atlas(A, 3, coords=X0, iterations=130)
    assert np.array_equal(ctx.force_atlas(A, 3, coords=X0, iterations=130), want)


@pytest.mark.parametrize("hook", [("GE_SMALL_GENERAL_ONLY", "1"), ("GE_SMALL_HANDOVER", "37"),
                                  ("GE_SMALL_HANDOVER", "0")])
def test_fa_small_kernel_handover(ctx, oracle, monkeypatch, hook):
    """The coarsest-level path is a domain-only kernel followed by the general
    kernel from the iteration it stopped at; force the general kernel from the
    start and a hand-over in the middle (coordinates and previous forces cross)."""
    monkeypatch.setenv(*hook)
    monkeypatch.setenv("GE_SMALL_MAX", "512")
    A = G.largest_component(G.rmat(300, 1500, seed=12))
    n = len(A[0]) - 1
    X0 = G.random_coords(n, 3, seed=3)
    want = oracle.force_atlas(A, 3, coords=X0, iterations=80)
    assert np.array_equal(ctx.force_atlas(A, 3, coords=X0, iterations=80), want)


@pytest.mark.parametrize("small_max", ["0", "512"])
def test_fa_small_kernel_out_of_domain_start(ctx, oracle, monkeypatch, small_max):
    """A coordinate below 2^-200 starts outside the shared-reciprocal domain: the
    domain-only kernel stops at once and the general kernel runs every step."""
    monkeypatch.setenv("GE_SMALL_MAX", small_max)
    A = G.largest_component(G.rmat(200, 900, seed=5))
    n = len(A[0]) - 1
    X0 = G.random_coords(n, 2, seed=4)
    X0[3, 1] = 1e-70
    want = oracle.force_atlas(A, 2, coords=X0, iterations=25)
    assert np.array_equal(ctx.force_atlas(A, 2, coords=X0, iterations=25), want)


@pytest.mark.parametrize("split", ["0", "1"])
@pytest.mark.parametrize("grp", ["1", "2", "4", "16", "32", "64"])
@pytest.mark.parametrize("n,dim", [(700, 3), (1400, 4), (2900, 2)])
def test_fa_grouped_repulsion(ctx, oracle, monkeypatch, grp, n, dim, split):
    """Small levels: G lanes per row, in-order group sums; one fused launch per
    iteration (fa_grouped_step) or repulsion + row kernels (GE_GRP_SPLIT=1)."""
    monkeypatch.setenv("GE_GRP_G", grp)
    if split == "1":
        monkeypatch.setenv("GE_GRP_SPLIT", "1")
    A = G.rmat(n, 6 * n, seed=n)
    X0 = G.random_coords(n, dim, seed=int(grp))
    want = oracle.force_atlas(A, dim, coords=X0, iterations=4)
    assert np.array_equal(ctx.force_atlas(A, dim, coords=X0, iterations=4), want)


@pytest.mark.parametrize("grp", ["0", "4", "16", "32", "64"])
@pytest.mark.parametrize("n,dim", [(4500, 3), (7000, 2), (3500, 4)])
def test_fa_grouped_stream(ctx, oracle, monkeypatch, grp, n, dim):
    """Mid-size levels (fa_grouped_stream): records streamed through LDS in tiles
    of 2048, G lanes per row (0 = default choice), neighbours read from X; a
    coordinate outside the exact-division domain sends one tile (and the rows
    next to it) through the general bodies."""
    if grp != "0":
        monkeypatch.setenv("GE_GRP_G", grp)
    A = G.with_degrees(G.rmat(n, 5 * n, seed=n), {17: 700}, seed=1)
    X0 = G.random_coords(n, dim, seed=int(grp) + 1)
    X0[2500, 0] = 1e-70
    want = oracle.force_atlas(A, dim, coords=X0, iterations=3)
    assert np.array_equal(ctx.force_atlas(A, dim, coords=X0, iterations=3), want)


def test_fa_small_level_graph_replay(ctx, oracle):
    """n = 127-ish coarsest level (fused grouped kernel, 64 lanes per row) over
    3000 iterations: captured-graph replay of the fused step, bit-exact."""
    A = G.largest_component(G.rmat(160, 700, seed=9))
    assert 64 < len(A[0]) - 1 <= 3072
    want = oracle.force_atlas(A, 3, iterations=3000, seed=77)
    assert np.array_equal(ctx.force_atlas(A, 3, iterations=3000, seed=77), want)


@pytest.mark.parametrize("n,dim,grp,its", [(300, 3, "0", 200), (700, 2, "0", 131),
                                            (1300, 4, "0", 128), (2900, 3, "32", 129),
                                            (1068, 3, "16", 140), (500, 1, "64", 257),
                                            (1068, 3, "nopack", 131), (97, 4, "0", 129),
                                            (1999, 2, "0", 128), (700, 3, "pack6", 131),
                                            (1068, 3, "pack4", 129), (1300, 1, "pack6", 128)])
def test_fa_persistent_small_level(ctx, oracle, monkeypatch, n, dim, grp, its):
    """Small levels with >= 128 iterations run every iteration in one launch
    (fa_grouped_persistent: resident blocks, grid barrier, coordinates in two
    alternating buffers); odd and even counts, G lanes per row.  At 64 lanes per
    row the rows are packed (packed_iteration: one adder wave, three producer
    waves; ragged last block, rows of degree above one chunk); "nopack" keeps one
    wave per row; "pack4" / "pack6" force 4 / 6 packed rows per block (4 is the
    default; 6 only where the blocks of 4 would not all be resident)."""
    monkeypatch.setenv("GE_PERSIST_REQUIRE", "1")
    if grp == "nopack":
        monkeypatch.setenv("GE_FA_PACKED", "0")
    elif grp.startswith("pack"):
        monkeypatch.setenv("GE_FA_PACK_ROWS", grp[4:])
    elif grp != "0":
        monkeypatch.setenv("GE_GRP_G", grp)
    A = G.rmat(n, 6 * n, seed=n + dim)
    X0 = G.random_coords(n, dim, seed=n)
    want = oracle.force_atlas(A, dim, coords=X0, iterations=its)
    assert np.array_equal(ctx.force_atlas(A, dim, coords=X0, iterations=its), want)


@pytest.mark.parametrize("pack", ["default", "4", "6"])
def test_fa_persistent_params_and_domain(ctx, oracle, monkeypatch, pack):
    """Non-default parameters (repel != 1, weights off) and a start outside the
    exact-division domain (the general bodies) in the persistent kernel.  With 6
    packed rows per block an out-of-domain block runs the general body twice over
    explicit row windows (rows r0..r0+3, then r0+4..r0+5; ge_fa.hip
    packed_iteration), so both packings are forced here."""
    monkeypatch.setenv("GE_PERSIST_REQUIRE", "1")
    if pack != "default":
        monkeypatch.setenv("GE_FA_PACK_ROWS", pack)
    A = G.largest_component(G.rmat(600, 3000, seed=8))
    n = len(A[0]) - 1
    X0 = G.random_coords(n, 3, seed=5)
    kw = dict(ks=0.2, ksmax=2.0, repel=1.5, attract=0.7, gravity=2.0, use_weights=0)
    want = oracle.force_atlas(A, 3, coords=X0, iterations=150, **kw)
    assert np.array_equal(ctx.force_atlas(A, 3, coords=X0, iterations=150, **kw), want)
    X0[7, 2] = 1e-70
    want = oracle.force_atlas(A, 3, coords=X0, iterations=130)
    assert np.array_equal(ctx.force_atlas(A, 3, coords=X0, iterations=130), want)


def test_fa_persistent_matches_graph_replay_long(ctx, monkeypatch):
    """C4's coarsest-level size (n ~ 1068, 64 lanes per row) over 20 000
    iterations: the persistent launch equals the per-iteration graph replay (which
    the oracle pins above) bit for bit."""
    A = G.largest_component(G.rmat(1400, 9000, seed=31))
    n = len(A[0]) - 1
    assert 900 < n <= 3072
    X0 = G.random_coords(n, 3, seed=12)
    monkeypatch.setenv("GE_PERSIST_REQUIRE", "1")
    got = ctx.force_atlas(A, 3, coords=X0, iterations=20000)
    monkeypatch.setenv("GE_NO_PERSIST", "1")
    assert np.array_equal(got, ctx.force_atlas(A, 3, coords=X0, iterations=20000))


def test_fa_coarsest_level_1e5_iterations(ctx, oracle):
    # the coarsest level runs the default 100000 iterations (src/embed.cpp:586);
    # chaos amplifies any op-order difference far beyond 1e-5 over that horizon
    A = G.largest_component(G.rmat(40, 120, seed=3))
    want = oracle.force_atlas(A, 3, iterations=100000, seed=555)
    got = ctx.force_atlas(A, 3, iterations=100000, seed=555)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("grp", ["0", "nopack", "16", "32", "pack6"])
def test_fa_coarsest_level_production_horizon(ctx, golden, monkeypatch, grp):
    """The coarsest level at its production size and horizon: an R-MAT LCC coarsened
    twice by partition(A, 0.125) (n = 1067, integer weights, self-loops), seeded
    random start, 100 000 iterations (src/embed.cpp:586) on the persistent
    grid-barrier kernel, against the oracle's run of the same 1e5 iterations
    (tests/golden/make_coarsest_1e5.py)."""
    monkeypatch.setenv("GE_PERSIST_REQUIRE", "1")
    if grp == "nopack":  # 64 lanes per row, one wave per row (grouped_iteration)
        monkeypatch.setenv("GE_FA_PACKED", "0")
    elif grp == "pack6":  # 6 packed rows per block (the default is 4 since round 6)
        monkeypatch.setenv("GE_FA_PACK_ROWS", "6")
    elif grp != "0":
        monkeypatch.setenv("GE_GRP_G", grp)
    g = golden("fa_coarsest_1e5")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    X = ctx.force_atlas(A, 3, iterations=int(g["iterations"]), seed=int(g["seed"]))
    assert np.array_equal(X, g["x"])


def test_fa_coarsest_level_shared_device(golden):
    """Three contexts run the coarsest level on one GPU at once, as the ranks of a
    one-GPU rehearsal do (every rank runs it as a replica): their persistent
    grids cannot all be resident together, so a late one either waits for the
    cooperative launch or times out at its barrier and reruns per iteration from
    the restored start.  Every result is still the oracle's."""
    import threading
    g = golden("fa_coarsest_1e5")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    its, seed = int(g["iterations"]), int(g["seed"])
    ctxs = [ge.Context(0) for _ in range(3)]
    out, errs = [None] * 3, []

    def run(k):
        try:
            out[k] = ctxs[k].force_atlas(A, 3, iterations=its, seed=seed)
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(e)

    th = [threading.Thread(target=run, args=(k,)) for k in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for c in ctxs:
        c.close()
    assert not errs, errs
    for X in out:
        assert np.array_equal(X, g["x"])


def test_fa_nondefault_params(ctx, oracle):
    A = G.erdos_renyi(1500, 0.004, seed=5)
    X0 = G.random_coords(1500, 3, seed=2)
    kw = dict(ks=0.2, ksmax=2.0, repel=1.5, attract=0.7, gravity=2.0, use_weights=0, tolerate=0.5)
    want = oracle.force_atlas(A, 3, coords=X0, iterations=4, **kw)
    assert np.array_equal(ctx.force_atlas(A, 3, coords=X0, iterations=4, **kw), want)
    want = oracle.force_atlas(A, 3, coords=X0, iterations=3, normalize=1)
    assert np.array_equal(ctx.force_atlas(A, 3, coords=X0, iterations=3, normalize=1), want)


def test_fa_edge_cases(ctx, oracle):
    one = (np.array([0, 0], np.int32), np.zeros(0, np.int32), np.zeros(0))
    X = ctx.force_atlas(one, 3, coords=np.array([[0.5, -0.25, 0.125]]), iterations=7)
    assert np.array_equal(X, oracle.force_atlas(one, 3, coords=np.array([[0.5, -0.25, 0.125]]),
                                                iterations=7))
    # isolated vertices + coincident points (distance clamped to eps)
    A = G.erdos_renyi(30, 0.05, seed=9)
    X0 = G.random_coords(30, 2, seed=3)
    X0[5] = X0[6]
    want = oracle.force_atlas(A, 2, coords=X0, iterations=10)
    assert np.array_equal(ctx.force_atlas(A, 2, coords=X0, iterations=10), want, equal_nan=True)
    assert ctx.force_atlas(one, 2, coords=np.zeros((1, 2)), iterations=0).shape == (1, 2)


def test_fa_fast_mode_tolerance(ctx, oracle):
    A = G.largest_component(G.rmat(3000, 24000, seed=11))
    m = len(A[0]) - 1
    X0 = G.random_coords(m, 3, seed=4)
    strict = ctx.force_atlas(A, 3, coords=X0, iterations=30)
    fast = ctx.force_atlas(A, 3, coords=X0, iterations=30, mode=ge.MODE_FAST)
    assert rel_err(fast, strict) < REL_TOL_FAST


@pytest.mark.parametrize("path", ["fused", "rows"])
def test_fa_plan_row_shards_compose(ctx, oracle, monkeypatch, path):
    """Two row shards stepping over a shared coordinate array (what each rank of
    the multi-GPU path runs between all-gathers) equal the unsharded iteration:
    small-level fused kernel, or the large-level kernels (repulsion row slots,
    row tiles, heavy-row segments inside a shard)."""
    torch = pytest.importorskip("torch")
    if path == "rows":
        monkeypatch.setenv("GE_STREAM_MAX", "0")
        monkeypatch.setenv("GE_ROWS_TILES", "1")
    A = G.largest_component(G.with_degrees(G.rmat(2600, 20000, seed=21), {4: 1300, 1700: 600},
                                           seed=2))
    n = len(A[0]) - 1
    X0 = G.random_coords(n, 3, seed=8)
    dev = torch.device("cuda:0")
    ip = torch.from_numpy(A[0].astype(np.int32)).to(dev)
    ix = torch.from_numpy(A[1].astype(np.int32)).to(dev)
    dx = torch.from_numpy(A[2]).to(dev)
    x = torch.from_numpy(X0.copy()).to(dev)
    y = torch.empty_like(x)
    half = n // 2
    plans = [ctx.fa_plan(n, len(A[1]), ip.data_ptr(), ix.data_ptr(), dx.data_ptr(), 3, lo, hi)
             for lo, hi in ((0, half), (half, n))]
    for _ in range(6):
        for p in plans:
            p.step(x.data_ptr(), y.data_ptr())
        x, y = y, x
    ctx.sync()
    want = oracle.force_atlas(A, 3, coords=X0, iterations=6)
    assert np.array_equal(x.cpu().numpy(), want)


@pytest.mark.parametrize("tiles", ["1", "0"])
def test_fa_plan_attract_on_supplied_repulsion(ctx, oracle, monkeypatch, tiles):
    """ge_fa_plan_attract: the attraction/update half of the iteration on a
    caller-supplied repulsion sum (the oracle's force rows with attract = 0 and
    gravity = 0, i.e. exactly the repulsion) equals one full oracle iteration;
    heavy rows as binade segments (tiles) or classed rows."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("GE_ROWS_TILES", tiles)
    A = G.with_degrees(G.rmat(5000, 20000, seed=31), {2: 3000, 9: 700}, seed=3)
    n = len(A[0]) - 1
    X0 = G.random_coords(n, 3, seed=12)
    deg = oracle.degrees(A)
    frep = oracle.fa_forces_rows(A, X0, deg, 0, n, attract=0.0, gravity=0.0)
    dev = torch.device("cuda:0")
    ip = torch.from_numpy(A[0].astype(np.int32)).to(dev)
    ix = torch.from_numpy(A[1].astype(np.int32)).to(dev)
    dx = torch.from_numpy(A[2]).to(dev)
    x = torch.from_numpy(X0.copy()).to(dev)
    f = torch.from_numpy(frep).to(dev)
    y = torch.empty_like(x)
    plan = ctx.fa_plan(n, len(A[1]), ip.data_ptr(), ix.data_ptr(), dx.data_ptr(), 3, 0, n)
    plan.attract(x.data_ptr(), f.data_ptr(), y.data_ptr())
    ctx.sync()
    plan.close()
    want = oracle.force_atlas(A, 3, coords=X0, iterations=1)
    assert np.array_equal(y.cpu().numpy(), want)


# --------------------------------------------------------------------------
# multilevel

def test_faml_golden(ctx, golden):
    g = golden("faml_rmat4096_l0")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    X = ctx.force_atlas_ml(A, (g["P_ip"], g["P_ix"]), g["vA"], g["cA"], g["rA"], 3,
                           iterations=100, seed=int(g["seed"]))
    assert np.array_equal(X, g["x_it100"])


def _block_partition(n, sizes, seed=0):
    """P_T with aggregates of the given sizes over a random permutation of 0..n-1,
    members listed ascending (as the partitioner emits them)."""
    assert sum(sizes) == n
    perm = np.random.RandomState(seed).permutation(n)
    ip = np.cumsum([0] + list(sizes)).astype(np.int32)
    ix = np.concatenate([np.sort(perm[ip[a]:ip[a + 1]]) for a in range(len(sizes))])
    return ip, ix.astype(np.int32)


@pytest.mark.parametrize("sizes", [
    [1, 2, 3, 5, 8, 13, 21, 34, 64, 9],            # packed 64-lane blocks
    [65, 100, 256, 3, 200],                         # 256-member packs
    [257, 1000, 4096, 17],                          # one aggregate per block, LDS-resident
    [5000, 300, 40, 1],                             # streamed (> 4096) path
])
def test_faml_size_classes(ctx, oracle, sizes):
    n = sum(sizes)
    A = G.submatrix(G.rmat(n, 6 * n, seed=len(sizes)), np.arange(n))
    PT = _block_partition(n, sizes, seed=n)
    vA = ge.vertex_of(PT)
    m = len(sizes)
    cA = G.random_coords(m, 3, seed=m)
    rA = np.random.RandomState(m).uniform(0.0, 0.6, m)
    it = 4 if n > 4000 else 12
    want = oracle.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=it, seed=31)
    got = ctx.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=it, seed=31)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("R,U,tiles,segs,repel", [
    (1, 1, "0", "1", 1.0), (1, 1, "1", "1", 1.0), (1, 1, "1", "0", 1.0), (1, 2, "1", "1", 1.0),
    (1, 4, "0", "1", 1.0), (2, 1, "1", "1", 1.0), (4, 1, "0", "1", 1.0), (1, 1, "1", "1", 1.5),
    (2, 1, "1", "1", 0.75)])
def test_faml_streamed_row_slots(ctx, oracle, monkeypatch, R, U, tiles, segs, repel):
    """Streamed path (faml_big_repulse / faml_big_edges) with 1, 2 and 4 row
    slots per lane (full and ragged items), repel = 1 and not, and hub rows longer
    than one 64-edge chunk;
    member rows tiled or classed (GE_ROWS_TILES), heavy member rows as stored-term
    segments + one chain wave per row, or whole rows on a side stream
    (GE_ROWS_SEGMENTS=0)."""
    monkeypatch.setenv("GE_ROWS_TILES", tiles)
    monkeypatch.setenv("GE_ROWS_SEGMENTS", segs)
    monkeypatch.setenv("GE_FAML_SYM", "0")  # the ordered-pair kernel (faml_big_repulse)
    monkeypatch.setenv("GE_FAML_R", str(R))
    monkeypatch.setenv("GE_FAML_U", str(U))
    sizes = [3000, 700, 2203, 90, 1]
    n = sum(sizes)
    A = G.with_hubs(G.rmat(n, 10 * n, seed=7), [(3, 2600), (40, 5000)], seed=R)
    assert np.diff(A[0]).max() > 4096
    PT = _block_partition(n, sizes, seed=3)
    vA = ge.vertex_of(PT)
    m = len(sizes)
    cA = G.random_coords(m, 3, seed=m)
    rA = np.random.RandomState(m).uniform(0.0, 0.6, m)
    want = oracle.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=5, seed=17, repel=repel)
    got = ctx.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=5, seed=17, repel=repel)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("dim", [3, 2])
def test_faml_early_heavy_row_chains(ctx, oracle, monkeypatch, dim):
    """Heavy member rows of >= kChainEarly (8 192) entries (ge_rows.hpp launch_rows):
    their segments and chains run on the side stream beside the tiles' launch, which
    takes the other heavy rows' segments; the short chains follow it.  Two early rows
    (~12 000 and ~9 000 entries) and a later heavy row (~5 000), tiles forced."""
    monkeypatch.setenv("GE_ROWS_TILES", "1")
    sizes = [12000, 3000, 2000, 300]
    n = sum(sizes)
    A = G.with_hubs(G.rmat(n, 8 * n, seed=23), [(5, 12000), (600, 9000), (40, 5000)], seed=dim)
    deg = np.diff(A[0])
    assert (deg >= 8192).sum() >= 2 and ((deg > 512) & (deg < 8192)).any()
    PT = _block_partition(n, sizes, seed=9)
    vA = ge.vertex_of(PT)
    m = len(sizes)
    cA = G.random_coords(m, dim, seed=m)
    rA = np.random.RandomState(m).uniform(0.0, 0.6, m)
    want = oracle.force_atlas_ml(A, PT, vA, cA, rA, dim, iterations=3, seed=29)
    got = ctx.force_atlas_ml(A, PT, vA, cA, rA, dim, iterations=3, seed=29)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("chain,dim,repel", [
    ("0", 3, 1.0), ("0", 3, 1.5), ("0", 3, 2.0 ** 70), ("1e9", 3, 1.0), ("", 3, 1.0),
    ("0", 2, 1.0), ("0", 4, 0.75), ("1e9", 4, 1.0)])
def test_faml_symmetric_sweeps(ctx, oracle, monkeypatch, chain, dim, repel):
    """faml_sym_repulse (ge_sym.hpp): every unordered pair once, row sums in the
    reference's order -- all aggregates as sweeps (chain 0), all as row blocks
    (1e9), the plan's own mix; repel = 2^70 forces the `/` path (outside the
    shared-reciprocal domain); ragged last tiles (sizes not multiples of 64),
    whole and one-member last tiles (320, 257), hub rows."""
    monkeypatch.setenv("GE_FAML_SYM", "1")
    if chain:
        monkeypatch.setenv("GE_FAML_SYM_CHAIN", chain)
    sizes = [2600, 320, 700, 257, 1031, 300, 90, 1]  # streamed: > 256 members
    n = sum(sizes)
    A = G.with_hubs(G.rmat(n, 10 * n, seed=11), [(3, 2000), (70, 3000)], seed=dim)
    PT = _block_partition(n, sizes, seed=5)
    vA = ge.vertex_of(PT)
    m = len(sizes)
    cA = G.random_coords(m, dim, seed=m)
    rA = np.random.RandomState(m).uniform(0.0, 0.6, m)
    want = oracle.force_atlas_ml(A, PT, vA, cA, rA, dim, iterations=6, seed=19, repel=repel)
    got = ctx.force_atlas_ml(A, PT, vA, cA, rA, dim, iterations=6, seed=19, repel=repel)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("dim", [2, 4])
def test_faml_dims(ctx, oracle, dim):
    A = G.largest_component(G.rmat(1500, 9000, seed=dim))
    PT = oracle.partition(A, 0.125)[0]
    vA = ge.vertex_of(PT)
    cA = G.random_coords(PT[2], dim, seed=1)
    rA = np.random.RandomState(2).uniform(0.1, 0.4, PT[2])
    want = oracle.force_atlas_ml(A, PT, vA, cA, rA, dim, iterations=20, seed=5)
    assert np.array_equal(ctx.force_atlas_ml(A, PT, vA, cA, rA, dim, iterations=20, seed=5),
                          want)


# --------------------------------------------------------------------------
# P^T A P and end-to-end embed

def test_ptap_golden(ctx, golden):
    g = golden("partition_rmat4096")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    for l in range(int(g["levels"])):
        PT = (g[f"P{l}_ip"], g[f"P{l}_ix"])
        C = ctx.ptap(A, PT)
        want = (g[f"A{l + 1}_ip"], g[f"A{l + 1}_ix"], g[f"A{l + 1}_dx"])
        for a, b in zip(C, want):
            assert np.array_equal(a, b)
        A = C


def test_ptap_nonunit_weights(ctx, oracle):
    A = G.largest_component(G.rmat(3000, 20000, seed=4))
    A = (A[0], A[1], np.random.RandomState(1).uniform(0.1, 2.0, len(A[1])))
    PT = oracle.partition(A, 0.2)[0]
    C = ctx.ptap(A, PT)
    for a, b in zip(C, oracle.ptap(A, PT)):
        assert np.array_equal(a, b)


def test_embed_c1_golden(ctx, golden):
    g = golden("embed_c1_er1000_d2")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    hier = ge.partition(A, 0.1)
    As = [A]
    for PT in hier:
        As.append(ctx.ptap(As[-1], PT))
    X = ctx.embed(As, hier, 2, seed=int(g["seed"]))
    assert np.array_equal(X, g["coords"])


def test_embed_rmat_vs_oracle(ctx, oracle):
    A = G.largest_component(G.rmat(6000, 50000, seed=12345))
    hier = ge.partition(A, 0.125)[:4]  # examples/embedder.cpp:189-192 truncation pattern
    As = [A]
    for PT in hier:
        As.append(ctx.ptap(As[-1], PT))
    X = ctx.embed(As, hier, 3, seed=9, base_iterations=20000)
    want = oracle.embed(As, hier, 3, seed=9, base_iterations=20000)
    assert np.array_equal(X, want)
    assert np.isfinite(X).all()


def test_faml_plan_device_resident_and_ranges(ctx, oracle):
    """ge_faml_plan_* (device pointers, the bench / multi-GPU path) on a full
    level and on two aggregate ranges that together cover it."""
    torch = pytest.importorskip("torch")
    A = G.largest_component(G.rmat(5000, 40000, seed=99))
    n = len(A[0]) - 1
    PT = oracle.partition(A, 0.125)[0]
    m = PT[2]
    vA = ge.vertex_of(PT)
    cA = G.random_coords(m, 3, seed=3)
    rA = np.random.RandomState(4).uniform(0.05, 0.3, m)
    want = oracle.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=25, seed=8)
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d = [T(A[0]), T(A[1]), T(A[2]), T(PT[0]), T(PT[1]), T(vA), T(cA), T(rA),
         T(ge.uniform_stream(8, n * 3))]
    ptr = [t.data_ptr() for t in d]
    for ranges in ([(0, m)], [(0, m // 3), (m // 3, m)]):
        X = torch.zeros((n, 3), dtype=torch.float64, device=dev)
        for rg in ranges:
            plan = ge.FamlPlan(ctx, n, ptr[0], ptr[1], ptr[2], PT[0], ptr[3], ptr[4], ptr[5], 3,
                               iterations=25, agg_range=rg)
            plan.run(ptr[6], ptr[7], ptr[8], X.data_ptr())
            ctx.sync()
            plan.close()
        assert np.array_equal(X.cpu().numpy(), want)


@pytest.mark.parametrize("world", [2, 3])
def test_faml_plan_aggregate_subsets_compose(ctx, oracle, world):
    """ge_faml_plan_create_subset with the multi-GPU assignment (LPT by cost),
    the ranks' plans run one after another on this GPU: together bit-exact."""
    torch = pytest.importorskip("torch")
    from ge_amd.dist import aggregate_cost, assign_aggregates
    A = G.with_hubs(G.largest_component(G.rmat(6000, 50000, seed=5)), [(0, 2500)], seed=1)
    n = len(A[0]) - 1
    PT = oracle.partition(A, 0.125)[0]
    m = PT[2]
    vA = ge.vertex_of(PT)
    cA = G.random_coords(m, 3, seed=6)
    rA = np.random.RandomState(7).uniform(0.05, 0.3, m)
    want = oracle.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=12, seed=9)
    owned, _ = assign_aggregates(aggregate_cost(PT[0], A[0], PT[1]), world)
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d = [T(A[0]), T(A[1]), T(A[2]), T(PT[0]), T(PT[1]), T(vA), T(cA), T(rA),
         T(ge.uniform_stream(9, n * 3))]
    ptr = [t.data_ptr() for t in d]
    X = torch.zeros((n, 3), dtype=torch.float64, device=dev)
    for aggs in owned:
        plan = ge.FamlPlan(ctx, n, ptr[0], ptr[1], ptr[2], PT[0], ptr[3], ptr[4], ptr[5], 3,
                           iterations=12, aggs=aggs)
        plan.run(ptr[6], ptr[7], ptr[8], X.data_ptr())
        ctx.sync()
        plan.close()
    assert np.array_equal(X.cpu().numpy(), want)


@pytest.mark.parametrize("weights", ["unit", "fractional"])
def test_modularity_device_matches_host(ctx, oracle, weights):
    """ge_modularity_device (integer atomics + host final sum) gives the host
    ge_modularity's bits, truncation of weights to int included."""
    A = G.largest_component(G.rmat(4000, 30000, seed=21))
    if weights == "fractional":
        A = (A[0], A[1], np.random.RandomState(3).uniform(0.2, 3.9, len(A[1])))
    for PT in oracle.partition(A, 0.125)[:3]:
        vA = ge.vertex_of(PT)
        m = PT[2]
        want = ge.modularity(A, vA, m)
        assert ctx.modularity(A, vA, m) == want
        A = ctx.ptap(A, PT)
