"""configs[4] (C5): the attraction pass on a 100M-vertex / 800M-draw R-MAT --
rocprof HBM-roofline report on the attraction SpMV.

All-pairs repulsion at n = 1e8 (1e16 pairs per iteration) is out of reach, so
this times the second half of the iteration alone (ge_fa_plan_attract: CSR
attraction in stored order + gravity + swing + update, bit-exact machinery of
the full path) on a SYNTHETIC repulsion sum: Frep[i][k] = (deg_i + 1) * 1e6 *
U(-1, 1), the scale of a repulsion over ~1e8 vertices.  Coordinates U(-1, 1)
(torch generator, seed 1).  Prints one JSON line; kernel times are HIP events
on the plan's stream (tile + heavy-segment + heavy-finish kernels, fork to join).

Algorithmic bytes per pass: 12*nnz + 52*n + 4 (int32 indptr /
indices, fp64 weights, read x, write x_next; fp64 d = 3).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))
import ge_amd as ge  # noqa: E402

HBM_PEAK_GBS = 8000.0


def bfs_order(ip, ix, n):
    """Cuthill-McKee order of a symmetric CSR on the device: new -> old ids."""
    dev = ip.device
    deg = torch.diff(ip).to(torch.int64)
    rank = torch.full((n,), -1, dtype=torch.int64, device=dev)
    src = int(torch.argmax(deg).item())
    rank[src] = 0
    frontier = torch.tensor([src], dtype=torch.int64, device=dev)
    nxt = 1
    big = torch.iinfo(torch.int64).max
    while frontier.numel():
        cnt = deg[frontier]
        tot = int(cnt.sum().item())
        if tot == 0:
            break
        starts = ip[frontier].to(torch.int64)
        off = torch.cumsum(cnt, 0) - cnt
        ent = torch.repeat_interleave(starts - off, cnt) + torch.arange(tot, device=dev)
        nb = ix[ent].to(torch.int64)
        del ent
        par = torch.repeat_interleave(rank[frontier], cnt)
        keep = rank[nb] < 0
        nb, par = nb[keep], par[keep]
        if nb.numel() == 0:
            break
        best = torch.full((n,), big, dtype=torch.int64, device=dev)
        best.scatter_reduce_(0, nb, par, reduce="amin")
        newv = torch.unique(nb)
        del nb, par
        key = best[newv] * n + newv
        newv = newv[torch.argsort(key)]
        del best, key
        rank[newv] = nxt + torch.arange(newv.numel(), device=dev)
        nxt += newv.numel()
        frontier = newv
    rest = torch.nonzero(rank < 0).flatten()
    rank[rest] = nxt + torch.arange(rest.numel(), device=dev)
    order = torch.empty(n, dtype=torch.int64, device=dev)
    order[rank] = torch.arange(n, device=dev)
    return order


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--draws", type=int, default=800_000_000)
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--relabel", choices=["none", "degree", "bfs"], default="none",
                    help="degree: vertices renumbered by descending degree (stable); bfs: "
                         "Cuthill-McKee order (breadth-first from the largest hub, each "
                         "level's vertices by their first parent's rank, then id; vertices "
                         "it does not reach after them in id order).  Rows and coordinates "
                         "permuted alike, each row's entry order kept; the pass's results "
                         "are the same values at permuted positions (checked against the "
                         "unpermuted pass)")
    a = ap.parse_args()
    dim = 3
    t0 = time.perf_counter()
    ctx = ge.Context(0)
    A = ctx.rmat_csr(a.n, a.draws, seed=a.seed)  # device generator (= the host arrays)
    n, nnz = len(A[0]) - 1, int(A[0][-1])
    print(f"R-MAT n={n} nnz={nnz} max deg={int(np.diff(A[0]).max())} "
          f"generated in {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
    dev = torch.device("cuda:0")
    ip = torch.from_numpy(A[0]).to(dev)
    ix = torch.from_numpy(A[1]).to(dev)
    dx = torch.from_numpy(A[2]).to(dev)
    deg = torch.diff(ip).to(torch.float64)
    del A
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    x = torch.rand(n, dim, dtype=torch.float64, device=dev, generator=g) * 2 - 1
    frep = (torch.rand(n, dim, dtype=torch.float64, device=dev, generator=g) * 2 - 1) * \
        ((deg + 1) * 1e6)[:, None]
    y = torch.empty_like(x)
    check = None
    if a.relabel != "none":
        t0 = time.perf_counter()
        plan = ctx.fa_plan(n, nnz, ip.data_ptr(), ix.data_ptr(), dx.data_ptr(), dim, 0, n)
        plan.attract(x.data_ptr(), frep.data_ptr(), y.data_ptr())
        ctx.sync()
        plan.close()
        if a.relabel == "degree":
            order = torch.sort(torch.diff(ip), descending=True, stable=True).indices  # new -> old
        else:
            order = bfs_order(ip, ix, n)
        new_id = torch.empty_like(order)
        new_id[order] = torch.arange(n, device=dev)
        dn = torch.diff(ip)[order]
        ip2 = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        ip2[1:] = torch.cumsum(dn, 0)
        src = torch.repeat_interleave(ip[:-1].to(torch.int64)[order] - ip2[:-1], dn) + \
            torch.arange(nnz, device=dev)
        ix = new_id[ix.to(torch.int64)[src]].to(torch.int32)
        dx = dx[src]
        del src
        ip = ip2.to(torch.int32)
        x, frep = x[order].contiguous(), frep[order].contiguous()
        check = y[order].clone()
        print(f"relabelled ({a.relabel}) in {time.perf_counter() - t0:.1f}s", file=sys.stderr,
              flush=True)
    t0 = time.perf_counter()
    plan = ctx.fa_plan(n, nnz, ip.data_ptr(), ix.data_ptr(), dx.data_ptr(), dim, 0, n)
    print(f"plan {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
    same = None
    if check is not None:  # first pass of a fresh plan on both sides
        plan.attract(x.data_ptr(), frep.data_ptr(), y.data_ptr())
        ctx.sync()
        same = bool(torch.equal(y, check))
    for _ in range(a.warmup):
        plan.attract(x.data_ptr(), frep.data_ptr(), y.data_ptr())
    ctx.sync()
    plan.set_profiling(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        plan.attract(x.data_ptr(), frep.data_ptr(), y.data_ptr())
    ctx.sync()
    wall = (time.perf_counter() - t0) / a.steps
    _, att_ms, launches = plan.kernel_ms()
    finite = bool(torch.isfinite(y).all().item())
    plan.close()
    ctx.close()
    bytes_alg = 12 * nnz + 52 * n + 4
    gbs = bytes_alg / (att_ms * 1e-3) / 1e9
    print(json.dumps({
        "workload": "C5 (BASELINE.json configs[4]) attraction pass: Graph500 R-MAT "
                    f"{a.n} ids, {a.draws} draws, d = 3, strict fp64, synthetic repulsion sums",
        "n": n, "nnz": nnz, "passes_per_s": 1e3 / att_ms, "edges_per_s": nnz * 1e3 / att_ms,
        "avg_pass_ms": att_ms, "wall_ms_per_pass": wall * 1e3, "launches": launches,
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_pass": bytes_alg},
        "relabel": a.relabel, "same_as_unpermuted": same, "finite": finite}), flush=True)


if __name__ == "__main__":
    main()
