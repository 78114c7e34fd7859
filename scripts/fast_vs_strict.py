#!/usr/bin/env python3
"""Drift of FAST mode against STRICT mode on the device, as a function of the
iteration count (the north star's 1e-5 relative bar).

    python scripts/fast_vs_strict.py --n 200000 --draws 1600000 --iters 100

Both modes start from the same reference-order random init; every `--every`
iterations the max-abs coordinate difference relative to max |x| is printed as
one JSON line.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200_000)
    ap.add_argument("--draws", type=int, default=1_600_000)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--every", type=int, default=10)
    ap.add_argument("--dim", type=int, default=3)
    args = ap.parse_args()
    import torch

    import ge_amd as ge
    dev = torch.device("cuda", 0)
    A = ge.rmat_csr(args.n, args.draws, seed=12345)
    n, nnz = len(A[0]) - 1, len(A[1])
    X0 = torch.from_numpy(ge.uniform_stream(12345, n * args.dim).reshape(n, args.dim)).to(dev)
    ip, ix, dx = (torch.from_numpy(a).to(dev) for a in A)
    ctx = ge.Context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    runs = {}
    for name, mode in (("strict", ge.MODE_STRICT), ("fast", ge.MODE_FAST)):
        plan = ctx.fa_plan(n, nnz, ip.data_ptr(), ix.data_ptr(), dx.data_ptr(), args.dim, 0, n,
                           mode=mode)
        runs[name] = [plan, X0.clone(), torch.empty_like(X0), 0.0]
    it = 0
    while it < args.iters:
        step = min(args.every, args.iters - it)
        for r in runs.values():
            plan, cur, nxt, _ = r
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(step):
                plan.step(cur.data_ptr(), nxt.data_ptr())
                cur, nxt = nxt, cur
            torch.cuda.synchronize(dev)
            r[1], r[2] = cur, nxt
            r[3] += time.perf_counter() - t0
        it += step
        s, f = runs["strict"][1], runs["fast"][1]
        rel = float((s - f).abs().max() / s.abs().max())
        print(json.dumps({"n": n, "nnz": nnz, "iteration": it, "rel_err": rel,
                          "strict_s_per_it": runs["strict"][3] / it,
                          "fast_s_per_it": runs["fast"][3] / it}), flush=True)
    for r in runs.values():
        r[0].close()
    ctx.close()


if __name__ == "__main__":
    main()
