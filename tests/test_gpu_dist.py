"""Multi-GPU inside libge (csrc/ge_dist.hip) through the C ABI.

* one rank on an RCCL communicator (ncclCommInitRank inside libge): the sharded
  entry points degenerate to the single-GPU ones and the collectives run;
* 2 and 3 ranks as separate processes sharing the box's one GPU, with the
  library's transport communicator (collectives staged through host memory and
  all-gathered over gloo): row-sharded forceAtlas (replica bound forced to 0),
  aggregate-sharded forceAtlasMultilevel, row-block P^T A P and the sharded
  embed must equal the single-GPU calls (and the oracle) bit for bit on every
  rank.  (RCCL itself cannot put two ranks on one device; the 8-GPU node runs
  the RCCL path in bench.py.)
The reference has no multi-GPU path; the expected results are its single-node
results (oracle restatement of include/forceatlas.hpp:89-574, src/embed.cpp:561-796).
"""
import os
import socket

import numpy as np
import pytest

import ge_amd as ge
import graphs as G

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs():
    A = G.largest_component(G.rmat(3000, 24000, seed=41))
    import oracle_lib
    oracle_lib.build()
    hier = oracle_lib.partition(A, 0.125)[:3]
    As = [A]
    for PT in hier:
        As.append(oracle_lib.ptap(As[-1], PT))
    PT = hier[0]
    m = PT[2]
    cA = G.random_coords(m, 3, seed=2)
    rA = np.random.RandomState(3).uniform(0.05, 0.4, m)
    X0 = G.random_coords(len(A[0]) - 1, 3, seed=4)
    return A, hier, As, PT, cA, rA, X0


def _run_all(api, inputs):
    A, hier, As, PT, cA, rA, X0 = inputs
    vA = ge.vertex_of(PT)
    out = {}
    out["fa"] = api.force_atlas(A, 3, coords=X0, iterations=6)
    out["fa_w"] = api.force_atlas(A, 3, coords=X0, iterations=3, repel=1.5, normalize=1)
    out["faml"] = api.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=12, seed=9)
    for l, P in enumerate(hier):
        C = api.ptap(As[l], P)
        out[f"ptap{l}_ip"], out[f"ptap{l}_ix"], out[f"ptap{l}_dx"] = C
    out["embed"] = api.embed(As, hier, 3, seed=11, base_iterations=1500, ml_iterations=25)
    return out


def _dist_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      GE_DIST_REPLICA_MAX="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = ge.Context(0)
    comm = ge.Comm(ctx, world, rank, backend="transport")
    assert comm.info() == (world, rank, False)
    res = _run_all(comm, _inputs())
    np.savez(out_path % rank, **res)
    comm.close()
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def single(ctx):
    return _run_all(ctx, _inputs())


def test_single_gpu_reference_matches_oracle(oracle, single):
    A, hier, As, PT, cA, rA, X0 = _inputs()
    assert np.array_equal(single["fa"], oracle.force_atlas(A, 3, coords=X0, iterations=6))
    vA = ge.vertex_of(PT)
    assert np.array_equal(single["faml"],
                          oracle.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=12, seed=9))
    assert np.array_equal(single["embed"],
                          oracle.embed(As, hier, 3, seed=11, base_iterations=1500,
                                       ml_iterations=25))


def test_rccl_single_rank(ctx, single):
    uid = ge.Comm.unique_id()
    comm = ge.Comm(ctx, 1, 0, backend="rccl", uid=uid)
    try:
        assert comm.info() == (1, 0, True)
        got = _run_all(comm, _inputs())
        for k, v in single.items():
            assert np.array_equal(got[k], v), k
        import torch
        x = torch.arange(30, dtype=torch.float64, device="cuda").reshape(10, 3)
        ref = x.clone()
        comm.allgather_coords(x.data_ptr(), 10, 3)
        torch.cuda.synchronize()
        assert torch.equal(x, ref)
    finally:
        comm.close()


@pytest.mark.parametrize("world", [2, 3])
def test_transport_ranks_match_single_gpu(tmp_path, single, world):
    import torch.multiprocessing as mp
    out = str(tmp_path / "r%d.npz")
    mp.start_processes(_dist_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        got = dict(np.load(out % r))
        for k, v in single.items():
            assert np.array_equal(got[k], v), (r, k)


def test_ptap_split_sort_path(ctx, oracle, monkeypatch):
    """The LSD (two-sort) P^T A P path used when (a, b, j) needs more than 64 key
    bits, forced on a small graph with fractional weights."""
    monkeypatch.setenv("GE_PTAP_SPLIT_SORT", "1")
    ip, ix, dx = G.largest_component(G.rmat(4000, 30000, seed=5))
    dx = np.random.RandomState(7).uniform(0.1, 3.0, len(dx))
    A = (ip, ix, dx)
    PT = oracle.partition((ip, ix, np.ones(len(ix))), 0.125)[0]
    for a, b in zip(ctx.ptap(A, PT), oracle.ptap(A, PT)):
        assert np.array_equal(a, b)


# --------------------------------------------------------------------------
# giant aggregates split by row tiles across ranks: every rank
# computes its tiles' rows (row blocks against all members, include/forceatlas.hpp:
# 394-410 ordered per row) and the split aggregates' rows are all-gathered after
# every iteration inside the plan.  GE_DIST_SPLIT_MIN forces the split.

_SPLIT_SIZES = [2600, 700, 257, 1031, 100, 90, 1]  # 100 members: 2 tiles, so with 3
# ranks one rank owns none of its rows and still joins every exchange


def _split_inputs():
    n = sum(_SPLIT_SIZES)
    A = G.with_hubs(G.rmat(n, 10 * n, seed=17), [(3, 2000), (70, 3000)], seed=3)
    perm = np.random.RandomState(5).permutation(n)
    ip = np.cumsum([0] + _SPLIT_SIZES).astype(np.int32)
    ix = np.concatenate([np.sort(perm[ip[a]:ip[a + 1]]) for a in range(len(_SPLIT_SIZES))])
    PT = (ip, ix.astype(np.int32), len(_SPLIT_SIZES), n)
    m = len(_SPLIT_SIZES)
    cA = G.random_coords(m, 3, seed=m)
    rA = np.random.RandomState(m).uniform(0.0, 0.6, m)
    return A, PT, cA, rA


def _split_worker(rank, world, port, out_path, sym):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GE_DIST_SPLIT_MIN="100",
                      GE_FAML_SYM=sym)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = ge.Context(0)
    comm = ge.Comm(ctx, world, rank, backend="transport")
    A, PT, cA, rA = _split_inputs()
    owner = ge.assign_aggregates_split(PT, A[0], world, 100)
    X = comm.force_atlas_ml(A, PT, ge.vertex_of(PT), cA, rA, 3, iterations=7, seed=13)
    np.savez(out_path % rank, X=X, owner=owner)
    comm.close()
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,sym", [(2, "1"), (3, "1"), (3, "0")])
def test_split_aggregates_match_single_gpu(tmp_path, ctx, oracle, world, sym):
    import torch.multiprocessing as mp
    A, PT, cA, rA = _split_inputs()
    vA = ge.vertex_of(PT)
    want = oracle.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=7, seed=13)
    assert np.array_equal(ctx.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=7, seed=13), want)
    out = str(tmp_path / "s%d.npz")
    mp.start_processes(_split_worker, args=(world, _free_port(), out, sym), nprocs=world,
                       join=True, start_method="spawn")
    for r in range(world):
        got = dict(np.load(out % r))
        assert list(got["owner"][:5]) == [-1] * 5  # the five largest were split
        assert np.array_equal(got["X"], want), r
