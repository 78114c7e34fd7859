"""Multi-rank forceAtlas on CPU (gloo, world_size 2 and 3): the row-sharded
driver used by bench.py (ge_amd.dist) with each rank's rows computed by the
oracle must reproduce the single-process iteration bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import graphs as G


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, A, X0, iters, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle_lib as O
    from ge_amd.dist import ShardedForceAtlas
    n, dim = X0.shape
    deg = O.degrees(A)
    state = {}

    def step_rows(cur, nxt, rb, re):
        if "fprev" not in state:
            state["fprev"] = np.zeros((re - rb, dim))
        xn = nxt.numpy()
        O.fa_step_rows(A, np.ascontiguousarray(cur.numpy()[:n]), deg, rb, re, state["fprev"],
                       xn, nthreads=1)

    drv = ShardedForceAtlas(n, world, rank, step_rows)
    cur = torch.zeros((drv.padded_rows, dim), dtype=torch.float64)
    cur[:n] = torch.from_numpy(X0)
    nxt = torch.zeros_like(cur)
    for _ in range(iters):
        drv.step(cur, nxt)
        cur, nxt = nxt, cur
    if rank == 0:
        np.save(out_path, cur[:n].numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_force_atlas_matches_single_process(oracle, tmp_path, world):
    A = G.largest_component(G.rmat(700, 5000, seed=17))
    n = len(A[0]) - 1
    X0 = G.random_coords(n, 3, seed=5)
    out = str(tmp_path / "x.npy")
    mp.start_processes(_worker, args=(world, _free_port(), A, X0, 7, out), nprocs=world,
                       join=True, start_method="spawn")
    got = np.load(out)
    want = oracle.force_atlas(A, 3, coords=X0, iterations=7)
    assert np.array_equal(got, want)


def test_row_shards_cover_exactly():
    from ge_amd.dist import row_shards
    for n in (1, 7, 1000, 1000001):
        for world in (1, 2, 3, 8):
            chunk, sh = row_shards(n, world)
            assert sh[0][0] == 0 and sh[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(sh, sh[1:]))
            assert chunk * world >= n


# --------------------------------------------------------------------------
# forceAtlasMultilevel sharded by aggregates (ge_amd.dist.assign_aggregates /
# allgather_members): each rank produces only its aggregates' member rows (here
# cut from the oracle's level result, standing in for its FamlPlan subset), the
# member all-gather must rebuild the whole level on every rank.

def _ml_worker(rank, world, port, PT, full, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ge_amd.dist import aggregate_cost, assign_aggregates, member_rows, allgather_members
    owned, _ = assign_aggregates(aggregate_cost(PT[0]), world)
    rows = [member_rows(PT[0], PT[1], o) for o in owned]
    X = torch.zeros(full.shape, dtype=torch.float64)
    mine = torch.as_tensor(rows[rank], dtype=torch.long)
    X[mine] = torch.from_numpy(full)[mine]
    allgather_members(X, rows, rank, world)
    np.save(out_path % rank, X.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_aggregate_sharded_level_gather(oracle, tmp_path, world):
    from ge_amd import vertex_of
    A = G.largest_component(G.rmat(2000, 14000, seed=23))
    PT = oracle.partition(A, 0.125)[0]
    vA = vertex_of(PT)
    m = PT[2]
    cA = G.random_coords(m, 3, seed=1)
    rA = np.random.RandomState(2).uniform(0.05, 0.3, m)
    full = oracle.force_atlas_ml(A, PT, vA, cA, rA, 3, iterations=10, seed=4)
    out = str(tmp_path / "x%d.npy")
    mp.start_processes(_ml_worker, args=(world, _free_port(), PT, full, out), nprocs=world,
                       join=True, start_method="spawn")
    for r in range(world):
        assert np.array_equal(np.load(out % r), full)


def test_assign_aggregates_partition_and_balance():
    from ge_amd.dist import aggregate_cost, assign_aggregates
    rs = np.random.RandomState(0)
    sizes = np.concatenate([rs.randint(1, 60, 5000), rs.randint(2000, 12000, 50)])
    pip = np.concatenate([[0], np.cumsum(sizes)])
    cost = aggregate_cost(pip)
    for world in (1, 2, 4, 8):
        owned, loads = assign_aggregates(cost, world)
        ids = np.sort(np.concatenate(owned))
        assert np.array_equal(ids, np.arange(len(sizes)))  # every aggregate exactly once
        assert all(np.all(np.diff(o) > 0) for o in owned)
        assert max(loads) <= cost.sum() / world + cost.max()  # LPT bound
        again, _ = assign_aggregates(cost, world)
        assert all(np.array_equal(a, b) for a, b in zip(owned, again))


def test_library_assign_aggregates_matches_harness():
    """libge's ge_assign_aggregates (the deal inside ge_force_atlas_ml_dist) gives
    every aggregate the rank the harness's LPT deal gives it (host-only call)."""
    import ge_amd as ge
    from ge_amd.dist import aggregate_cost, assign_aggregates
    A = G.largest_component(G.rmat(3000, 20000, seed=3))
    import oracle_lib as O
    O.build()
    PT = O.partition(A, 0.125)[0]
    for world in (1, 2, 3, 8):
        owned, _ = assign_aggregates(aggregate_cost(PT[0], A[0], PT[1]), world)
        want = np.empty(PT[2], dtype=np.int32)
        for r, o in enumerate(owned):
            want[o] = r
        assert np.array_equal(ge.assign_aggregates(PT, A[0], world), want)
        owned, _ = assign_aggregates(aggregate_cost(PT[0]), world)
        for r, o in enumerate(owned):
            want[o] = r
        assert np.array_equal(ge.assign_aggregates(PT, None, world), want)


def test_library_row_shard_matches_harness():
    import ge_amd as ge
    from ge_amd.dist import row_shards
    for n in (1, 7, 1000, 1000001):
        for world in (1, 2, 3, 8):
            chunk, sh = row_shards(n, world)
            for r in range(world):
                assert ge.row_shard(n, world, r) == (sh[r][0], sh[r][1], chunk)
