"""Row-sharded forceAtlas across ranks (one process per GPU).

forceAtlas (include/forceatlas.hpp:146-270) computes every vertex's new
position from ALL positions of the previous iteration, so the iteration shards
by rows: rank r owns rows [r*chunk, (r+1)*chunk) (the last shard may be short),
computes them against the full coordinate array, and one all-gather of the
fp64 coordinate array per iteration re-assembles it (backend "nccl" = RCCL over
xGMI on MI355X; "gloo" on CPU for the tests).  Nothing else is exchanged: the
global swing/traction sums are dead in the reference (:228, :242).

The coordinate buffers are padded to world*chunk rows so every rank's block has
the same size; padding rows are never read (the kernels iterate j < n).
"""


def row_shards(n, world):
    chunk = (n + world - 1) // world
    return chunk, [(min(n, r * chunk), min(n, (r + 1) * chunk)) for r in range(world)]


def allgather_rows(x_full, chunk, rank, world):
    """In-place all-gather of the per-rank row blocks of x_full (world*chunk rows)."""
    if world == 1:
        return
    import torch.distributed as dist
    # a separate send buffer keeps the collective out-of-place (chunk x d fp64)
    mine = x_full[rank * chunk:(rank + 1) * chunk].clone()
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(x_full, mine)
    else:  # gloo: list form, staged through host memory for device tensors
        host = x_full.cpu() if x_full.is_cuda else x_full
        dist.all_gather(list(host.split(chunk)), mine.cpu())
        if x_full.is_cuda:
            x_full.copy_(host)


class ShardedForceAtlas:
    """Drives iterations: step_rows(cur, nxt, rb, re) computes rows [rb, re) of
    nxt from cur (device plan or any stand-in), then the rows are all-gathered."""

    def __init__(self, n, world, rank, step_rows):
        self.n, self.world, self.rank = n, world, rank
        self.chunk, shards = row_shards(n, world)
        self.rb, self.re = shards[rank]
        self.step_rows = step_rows

    @property
    def padded_rows(self):
        return self.chunk * self.world

    def step(self, cur, nxt):
        self.step_rows(cur, nxt, self.rb, self.re)
        allgather_rows(nxt, self.chunk, self.rank, self.world)


# ---------------------------------------------------------------------------
# forceAtlasMultilevel across ranks: aggregates never exchange
# data during the 100 iterations (include/forceatlas.hpp:454, :462 read only
# the frozen coarse coordinates), so a level shards by aggregates with no
# per-iteration collective.  One all-gather of the members' coordinates per
# level call reassembles the fine coordinate array.

def aggregate_cost(pt_indptr, indptr=None, pt_indices=None):
    """Per-aggregate work of one iteration: s(s-1) in-aggregate pairs plus the
    members' CSR entries (when the fine CSR is given)."""
    import numpy as np
    pip = np.asarray(pt_indptr, dtype=np.int64)
    s = np.diff(pip).astype(np.float64)
    cost = s * (s - 1)
    if indptr is not None:
        deg = np.diff(np.asarray(indptr, dtype=np.int64)).astype(np.float64)
        cost = cost + np.add.reduceat(deg[np.asarray(pt_indices)], pip[:-1]) * (s > 0)
    return cost


def assign_aggregates(cost, world):
    """Longest-processing-time list scheduling: aggregates in descending cost go
    to the least-loaded rank (ties: lowest rank).  Deterministic; returns the
    per-rank id lists (ascending) and loads."""
    import heapq
    import numpy as np
    cost = np.asarray(cost, dtype=np.float64)
    order = np.lexsort((np.arange(len(cost)), -cost))
    heap = [(0.0, r) for r in range(world)]
    owned = [[] for _ in range(world)]
    for a in order:
        load, r = heapq.heappop(heap)
        owned[r].append(int(a))
        heapq.heappush(heap, (load + float(cost[a]), r))
    loads = [float(cost[o].sum()) if o else 0.0 for o in owned]
    return [np.array(sorted(o), dtype=np.int32) for o in owned], loads


def member_rows(pt_indptr, pt_indices, aggs):
    """Fine vertex ids of the members of `aggs`, in aggregate then P_T order."""
    import numpy as np
    pip = np.asarray(pt_indptr)
    pix = np.asarray(pt_indices)
    if len(aggs) == 0:
        return np.zeros(0, dtype=np.int64)
    return np.concatenate([pix[pip[a]:pip[a + 1]] for a in aggs]).astype(np.int64)


def allgather_members(X, rows_per_rank, rank, world):
    """Every rank computed X[rows_per_rank[rank]]; afterwards every rank holds all
    rows.  Rows are packed, all-gathered with equal (padded) blocks, and scattered
    back -- copies only, so the bits are unchanged."""
    if world == 1:
        return
    import torch
    import torch.distributed as dist
    counts = [len(r) for r in rows_per_rank]
    width = max(counts)
    dev = X.device
    idx = [torch.as_tensor(r, dtype=torch.long, device=dev) for r in rows_per_rank]
    send = torch.zeros((width, X.shape[1]), dtype=X.dtype, device=dev)
    send[:counts[rank]] = X.index_select(0, idx[rank])
    recv = torch.empty((world * width, X.shape[1]), dtype=X.dtype, device=dev)
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(recv, send)
    else:  # gloo, staged through host memory for device tensors
        host = recv.cpu()
        dist.all_gather(list(host.split(width)), send.cpu())
        recv.copy_(host)
    for r in range(world):
        if r != rank and counts[r]:
            X.index_copy_(0, idx[r], recv[r * width:r * width + counts[r]])
