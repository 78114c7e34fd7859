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
    else:  # gloo: list form
        parts = list(x_full.split(chunk))
        dist.all_gather(parts, mine)


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
