"""Device partition (graph-embed_amd/csrc/ge_partition_dev.hip) against the oracle.

partition::partition (src/partitioner.cpp:1550-1893) is deterministic and the
P_T arrays are integer data, so the bar is bit-exact: the same number of levels,
the same rows / columns and the same indptr / indices arrays as
oracle.partition (oracle/ge_oracle.cpp, a line-cited restatement of the
reference loop), on the golden fixture, seeded R-MAT / ER graphs, every option
of the signature, non-unit integer weights, and the C3 graph (configs[2]: the
LCC of the 1M-id R-MAT) through the committed oracle digest
tests/golden/partition_c3_digest.json (tests/golden/make_partition_digest.py).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import ge_amd as ge
import graphs as G

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(autouse=True)
def device_required(monkeypatch):
    """A device-path failure of any kind (the list pool's capacity limit included)
    fails the test instead of silently falling back to the host path."""
    monkeypatch.setenv("GE_PARTITION_DEVICE_REQUIRE", "1")


def same(hg, ho):
    assert len(hg) == len(ho)
    for a, b in zip(hg, ho):
        assert a[2:] == b[2:]
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_partition_device_golden(ctx, golden):
    g = golden("partition_rmat4096")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    hg = ctx.partition(A, 0.125)  # tests/golden/make_golden.py: partition(C, 0.125)
    assert len(hg) == int(g["levels"])
    for l, PT in enumerate(hg):
        assert np.array_equal(PT[0], g[f"P{l}_ip"]) and np.array_equal(PT[1], g[f"P{l}_ix"])


def test_partition_device_er_c1(ctx, golden):
    g = golden("embed_c1_er1000_d2")
    A = (g["A_ip"], g["A_ix"], g["A_dx"])
    hg = ctx.partition(A, 0.1)
    assert len(hg) == int(g["levels"])
    for l, PT in enumerate(hg):
        assert np.array_equal(PT[0], g[f"P{l}_ip"]) and np.array_equal(PT[1], g[f"P{l}_ix"])


@pytest.mark.parametrize("n,draws,cf", [(2000, 16000, 0.125), (4096, 40000, 0.125),
                                        (1500, 9000, 0.3), (9000, 70000, 0.125),
                                        (30000, 150000, 0.1)])
def test_partition_device_rmat(ctx, oracle, n, draws, cf):
    A = G.largest_component(G.rmat(n, draws, seed=n))
    same(ctx.partition(A, cf), oracle.partition(A, cf))


@pytest.mark.parametrize("mode", ["GE_PARTITION_NO_PATCH", "GE_PARTITION_FULL_SCANS"])
def test_partition_device_alternative_paths(ctx, oracle, monkeypatch, mode):
    """The device partition's two exact shortcuts switched off one at a time: every
    dirty list rebuilt instead of hub lists patched in place, and every untouched
    vertex rescanned in every pass instead of the recorded-bound skips (DESIGN.md 5,
    partition rounds).  Same hierarchy as the oracle either way."""
    monkeypatch.setenv(mode, "1")
    A = G.largest_component(G.rmat(30000, 240000, seed=17))
    same(ctx.partition(A, 0.125), oracle.partition(A, 0.125))


def test_partition_device_er_and_components(ctx, oracle):
    # several components (no LCC) and an ER graph: ties everywhere
    A = G.rmat(3000, 6000, seed=11)
    same(ctx.partition(A, 0.2), oracle.partition(A, 0.2))
    A = G.erdos_renyi(2000, 0.004, seed=3)
    same(ctx.partition(A, 0.125), oracle.partition(A, 0.125))


def test_partition_device_options(ctx, oracle):
    A = G.largest_component(G.rmat(1200, 8000, seed=77))
    for kw in (dict(positive_merging=False), dict(matching_iterations=1),
               dict(matching_iterations=3), dict(stall=0.99)):
        hg = ctx.partition(A, 0.2, **kw)
        ho = oracle.partition(A, 0.2, positive_merging=kw.get("positive_merging", True),
                              stall=kw.get("stall", 1.0),
                              matching=kw.get("matching_iterations", 2))
        same(hg, ho)


def test_partition_device_integer_weights_and_self_loops(ctx, oracle):
    ip, ix, _ = G.largest_component(G.rmat(3000, 20000, seed=5))
    n = len(ip) - 1
    rows = np.repeat(np.arange(n), np.diff(ip))
    lo, hi = np.minimum(rows, ix), np.maximum(rows, ix)
    w = ((lo.astype(np.int64) * 7919 + hi * 104729) % 9 + 1).astype(np.float64)  # symmetric
    A = (ip, ix, w)
    same(ctx.partition(A, 0.125), oracle.partition(A, 0.125))
    # diagonal entries (count in alpha and T, not in the adjacency: :1569-1573)
    rr = np.arange(0, n, 7)
    M = {(int(r), int(c)): float(x) for r, c, x in zip(rows, ix, w)}
    for r in rr:
        M[(int(r), int(r))] = 3.0
    keys = sorted(M)
    r2 = np.array([k[0] for k in keys], np.int32)
    A2 = (np.concatenate([[0], np.cumsum(np.bincount(r2, minlength=n))]).astype(np.int32),
          np.array([k[1] for k in keys], np.int32), np.array([M[k] for k in keys]))
    same(ctx.partition(A2, 0.125), oracle.partition(A2, 0.125))


def test_partition_device_fractional_weights_take_host_path(ctx, oracle):
    ip, ix, _ = G.largest_component(G.rmat(1500, 9000, seed=9))
    rows = np.repeat(np.arange(len(ip) - 1), np.diff(ip))
    w = 0.5 + ((np.minimum(rows, ix) + np.maximum(rows, ix)) % 5) * 0.25
    A = (ip, ix, w)
    same(ctx.partition(A, 0.125), oracle.partition(A, 0.125))


def test_partition_device_matches_host_path_100k(ctx):
    A = ge.largest_component(ge.rmat_csr(150000, 1000000, seed=7))
    same(ctx.partition(A, 0.125), ge.partition(A, 0.125))


def _check_digest(ctx, name):
    with open(os.path.join(HERE, "golden", name)) as f:
        want = json.load(f)
    # the device R-MAT + LCC (equal to the host arrays, tests/test_gpu_graph.py)
    L = ctx.rmat_csr(want["n_ids"], want["draws"], seed=want["seed"], lcc=True)
    assert len(L[0]) - 1 == want["lcc_n"] and len(L[1]) == want["lcc_nnz"]
    hg = ctx.partition(L, want["cf"])
    assert [h[2] for h in hg] == want["rows"]
    dig = hashlib.sha256()
    for l, (ip, ix, _, _) in enumerate(hg):
        ipb = np.ascontiguousarray(ip, dtype=np.int32).tobytes()
        ixb = np.ascontiguousarray(ix, dtype=np.int32).tobytes()
        if "level_sha256" in want:  # the first differing level, if any
            assert hashlib.sha256(ipb + ixb).hexdigest() == want["level_sha256"][l], l
        dig.update(ipb)
        dig.update(ixb)
    assert dig.hexdigest() == want["sha256"]


def test_partition_device_c3_digest(ctx):
    """configs[2]: LCC of the R-MAT(1M ids, 8M draws, seed 12345) -- the oracle's
    hierarchy digest, committed (generator: tests/golden/make_partition_digest.py)."""
    _check_digest(ctx, "partition_c3_digest.json")


def test_partition_device_c4_digest(ctx):
    """configs[3] (the headline): LCC of the R-MAT(10M ids, 80M draws, seed 12345),
    4.39M vertices, 9 969 rounds -- the oracle's hierarchy digest (orc_partition_flat:
    the reference loop over unordered entry lists, 1 327 s on 5 threads here; it
    reproduced the std::map oracle's C3 digest in the same run; make_partition_digest.py
    --flat).  The library's host path (csrc/ge_partition.cpp) gave the same digest in
    round 4."""
    _check_digest(ctx, "partition_c4_digest.json")
