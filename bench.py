#!/usr/bin/env python3
"""ForceAtlas iteration benchmark on MI355X (BASELINE.json metric).

Workload (config.workload): BASELINE.json configs[1] ("C2") -- single-level
3-D forceAtlas on a 1,000,000-vertex Graph500 R-MAT (8,000,000 draws,
symmetrised, ~15M stored entries).  One step = one full forceAtlas iteration
(include/forceatlas.hpp:146-270): all-pairs repulsion + CSR attraction +
gravity + swing/speed update for every vertex, in STRICT mode (bit-exact with
the reference's serial fp64 op order).  Inputs are resident in HBM before the
timed region.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
contiguous row shards, one RCCL all-gather of the fp64 coordinate array per
iteration (the only exchange the iteration has).  The problem size is fixed, so
"scaling" is "strong".  value = iterations/s of the whole job.

Also reported: edges/s (= nnz x iterations/s), the roofline of the dominant
kernel (repulsion) from HIP events on the launching stream, the attraction
kernel's HBM roofline, and a CPU baseline (the oracle, rank 0, N = 1 only).
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))

METRIC = "ForceAtlas iterations/sec + edges/sec, 3-D embed, 10M-vtx R-MAT @1/2/4/8 GPU"
FP64_PEAK_TFLOPS = 78.6  # MI355X dense FP64 (matrix = vector) peak, spec
HBM_PEAK_GBS = 8000.0    # MI355X HBM3E peak, MI355X_MICROARCH.md
FLOPS_PER_PAIR = 26      # (7d+5) at d=3, SURVEY.md 8(d)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--draws", type=int, default=8_000_000)
    ap.add_argument("--dim", type=int, default=3)
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--mode", choices=["strict", "fast"], default="strict")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def pmc_traffic_per_launch(kernel_prefix):
    """HBM bytes per launch of a kernel from the committed rocprofv3 PMC passes
    (profiles/*/pmc_fetch*.csv, pmc_write*.csv).  gfx950 correction from
    MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of a wide coalesced
    read -> bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024."""
    def read(pattern, counter):
        files = sorted(glob.glob(os.path.join(REPO, "profiles", "*", pattern)))
        if not files:
            return None
        import csv
        vals = []
        with open(files[-1]) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") == counter and row.get("Kernel_Name", "").find(
                        kernel_prefix) >= 0:
                    vals.append(float(row["Counter_Value"]))
        return (sum(vals) / len(vals), files[-1]) if vals else None
    f = read("pmc_fetch*.csv", "FETCH_SIZE")
    w = read("pmc_write*.csv", "WRITE_SIZE")
    if not f or not w:
        return None, None
    return (2.0 * f[0] + w[0]) * 1024.0, [os.path.relpath(f[1], REPO), os.path.relpath(w[1], REPO)]


def cpu_baseline(A, X0, dim, seconds, rank):
    """Oracle (CPU restatement of the reference OpenMP loop) on a bounded sample:
    the force rows of one iteration for a contiguous block of rows, scaled to a
    full iteration (per-row cost is n pairs + deg(i) edges: uniform)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    oracle_lib.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    n = len(A[0]) - 1
    deg = oracle_lib.degrees(A)
    rb = n // 2
    rows = 256
    t0 = time.perf_counter()
    oracle_lib.fa_forces_rows(A, X0, deg, rb, rb + rows, nthreads=threads)
    t = time.perf_counter() - t0
    rows = int(min(n - rb, max(rows, rows * seconds / max(t, 1e-3))))
    t0 = time.perf_counter()
    oracle_lib.fa_forces_rows(A, X0, deg, rb, rb + rows, nthreads=threads)
    t = time.perf_counter() - t0
    per_iter = t * n / rows
    log(rank, f"cpu baseline: {rows} rows in {t:.2f}s on {threads} threads -> {per_iter:.1f}s/iter")
    return {"value": 1.0 / per_iter, "unit": "iterations/s", "cores": threads, "kind": "port",
            "sample": f"oracle forceAtlas force pass for rows [{rb},{rb + rows}) of one iteration "
                      f"({rows} of {n} rows, {t:.1f}s, OpenMP {threads} threads), "
                      f"scaled by n/rows to one full iteration",
            "seconds_per_iteration": per_iter}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    import ge_amd as ge

    # ---- synthetic input (identical on every rank: counter-based generator) ----
    t0 = time.perf_counter()
    A = ge.rmat_csr(args.n, args.draws, seed=args.seed)
    n, nnz = len(A[0]) - 1, len(A[1])
    X0 = ge.uniform_stream(args.seed, n * args.dim).reshape(n, args.dim)  # ref init order
    log(rank, f"R-MAT n={n} nnz={nnz} generated in {time.perf_counter() - t0:.1f}s")

    from ge_amd.dist import ShardedForceAtlas
    drv = ShardedForceAtlas(n, world, rank, None)
    npad, rb, re = drv.padded_rows, drv.rb, drv.re
    ip = torch.from_numpy(A[0]).to(dev)
    ix = torch.from_numpy(A[1]).to(dev)
    dx = torch.from_numpy(A[2]).to(dev)
    xa = torch.zeros((npad, args.dim), dtype=torch.float64, device=dev)
    xa[:n] = torch.from_numpy(X0).to(dev)
    xb = torch.zeros_like(xa)

    ctx = ge.Context(local)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    mode = ge.MODE_FAST if args.mode == "fast" else ge.MODE_STRICT
    plan = ctx.fa_plan(n, nnz, ip.data_ptr(), ix.data_ptr(), dx.data_ptr(), args.dim, rb, re,
                       mode=mode)

    drv.step_rows = lambda cur, nxt, rb_, re_: plan.step(cur.data_ptr(), nxt.data_ptr())
    step = drv.step

    cur, nxt = xa, xb
    for _ in range(args.warmup):
        step(cur, nxt)
        cur, nxt = nxt, cur
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    plan.set_profiling(True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(cur, nxt)
        cur, nxt = nxt, cur
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    rep_ms, att_ms, launches = plan.kernel_ms()
    finite = bool(torch.isfinite(cur[:n]).all().item())

    its = args.steps / elapsed
    rows = re - rb
    pairs = rows * (n - 1)
    rep_tflops = FLOPS_PER_PAIR * pairs / (rep_ms * 1e-3) / 1e12 if rep_ms > 0 else 0.0
    attr_bytes = 12 * nnz * rows / n + 52 * rows + 4  # SURVEY 8(d) B_attr, this rank's rows
    att_gbs = attr_bytes / (att_ms * 1e-3) / 1e9 if att_ms > 0 else 0.0
    traffic, traffic_src = pmc_traffic_per_launch("fa_repulse")
    att_traffic, _ = pmc_traffic_per_launch("fa_attract_update")

    result = {
        "metric": METRIC,
        "value": its,
        "unit": "iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": "C2 (BASELINE.json configs[1]): single-level 3-D forceAtlas iteration, "
                        f"Graph500 R-MAT n={n}, {args.draws} draws, nnz={nnz}, {args.mode} fp64",
            "n": n, "nnz": nnz, "dim": args.dim, "mode": args.mode,
            "parallelism": f"rows{world}" + ("+allgather" if world > 1 else ""),
        },
        "edges_per_s": nnz * its,
        "pair_interactions_per_s": n * (n - 1) * its,
        "finite": finite,
        "roofline": {
            "kernel": "fa_repulse_%s (all-pairs repulsion, fp64)" % args.mode,
            "bound": "mfma",
            "pipe": "fp64 VALU; priced against the dense FP64 peak (78.6 TFLOP/s, spec), "
                    "which MI355X's FP64 matrix and vector pipes share",
            "achieved": rep_tflops,
            "peak": FP64_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": rep_tflops / FP64_PEAK_TFLOPS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "flops_per_launch": FLOPS_PER_PAIR * pairs,
            "avg_launch_ms": rep_ms,
            "launches": launches,
        },
        "roofline_attraction": {
            "kernel": "fa_attract_update_strict (CSR attraction + gravity + update)",
            "bound": "hbm",
            "achieved": att_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": att_gbs / HBM_PEAK_GBS,
            "traffic": att_traffic,
            "algorithmic_bytes_per_launch": attr_bytes,
            "avg_launch_ms": att_ms,
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(A, X0, args.dim, args.cpu_baseline_seconds, rank)
        result["vs_cpu_baseline"] = its / result["cpu_baseline"]["value"]
    plan.close()
    ctx.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
