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
    ap.add_argument("--workload", choices=["c2", "c3", "c4"], default="c2",
                    help="c2: single-level forceAtlas (configs[1]); c3: multilevel level-0 "
                         "forceAtlasMultilevel on the R-MAT LCC hierarchy (configs[2]); c4: the "
                         "same on the 10M-vertex R-MAT (configs[3]; host partition takes minutes)")
    ap.add_argument("--levels", type=int, default=4)
    ap.add_argument("--partition-cache", default="",
                    help="c3/c4: directory caching the host partition hierarchy")
    ap.add_argument("--ml-iterations", type=int, default=100)
    ap.add_argument("--sweep-slots", action="store_true",
                    help="c3: also time the streamed path's row-slot / partner variants")
    ap.add_argument("--end-to-end", action="store_true",
                    help="c3: also time partition::embed over the whole hierarchy")
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def pmc_traffic_per_launch(kernel_prefix, workload):
    """HBM bytes per step of the kernels whose names contain kernel_prefix (summed
    over distinct kernels, averaged over launches) from the committed rocprofv3 PMC passes of
    the same workload (profiles/*/pmc_fetch_<workload>*.csv, pmc_write_<...>.csv).  gfx950 correction from
    MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of a wide coalesced
    read -> bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024."""
    def read(pattern, counter):
        import csv
        # newest round directory first; the first file that traced this kernel wins
        for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*", pattern)), reverse=True):
            vals = {}  # per kernel name (one step may launch several matching kernels)
            with open(path) as f:
                for row in csv.DictReader(f):
                    name = row.get("Kernel_Name", "")
                    if row.get("Counter_Name") == counter and name.find(kernel_prefix) >= 0:
                        vals.setdefault(name, []).append(float(row["Counter_Value"]))
            if vals:
                return sum(sum(v) / len(v) for v in vals.values()), path
        return None
    f = read(f"pmc_fetch_{workload}*.csv", "FETCH_SIZE")
    w = read(f"pmc_write_{workload}*.csv", "WRITE_SIZE")
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


def cpu_baseline_ml(L, PT, vA, cA, rA, dim, seconds, rank):
    """Oracle forceAtlasMultilevel on a bounded sample of aggregates (every k-th
    aggregate), 1 iteration, scaled by the pair+edge cost of the full level."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    oracle_lib.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    pip, pix = np.asarray(PT[0]), np.asarray(PT[1])
    s = np.diff(pip).astype(np.float64)
    deg = np.diff(np.asarray(L[0])).astype(np.float64)
    row_edges = np.add.reduceat(deg[pix], pip[:-1]) if len(pix) else np.zeros(len(s))
    cost = s * (s - 1) + row_edges
    def run(stride):
        sel = np.arange(0, len(s), stride)
        sizes = np.diff(pip)[sel]
        sip = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
        six = np.concatenate([pix[pip[a]:pip[a + 1]] for a in sel]).astype(np.int32)
        t0 = time.perf_counter()
        oracle_lib.force_atlas_ml(L, (sip, six), vA, cA, rA, dim, iterations=1, seed=1,
                                  nthreads=threads)
        return time.perf_counter() - t0, cost[sel].sum()
    stride = 64
    t, c = run(stride)
    stride = max(1, int(stride * t / seconds)) if t > 0 else 1
    t, c = run(stride)
    per_iter = t * cost.sum() / c
    log(rank, f"cpu baseline (multilevel): stride {stride}, {t:.2f}s on {threads} threads "
              f"-> {per_iter:.2f}s/iteration")
    return {"value": 1.0 / per_iter, "unit": "iterations/s", "cores": threads, "kind": "port",
            "sample": f"oracle forceAtlasMultilevel, 1 iteration over every {stride}-th aggregate "
                      f"of level 0 ({t:.1f}s, OpenMP {threads} threads), scaled by the "
                      f"pair+edge cost of the whole level",
            "seconds_per_iteration": per_iter}


def partition_levels(L, args):
    """partition(L, 0.125)[:levels] (host, bit-exact).  With --partition-cache DIR
    the hierarchy is stored keyed by the generator parameters and a digest of the
    LCC arrays, and reloaded when both match (the partitioner is deterministic;
    the cache only skips its minutes of host time at configs[3])."""
    import ge_amd as ge
    import hashlib
    key = None
    if args.partition_cache:
        h = hashlib.sha1()
        for a in L[:2]:
            h.update(np.ascontiguousarray(a).view(np.uint8))
        key = os.path.join(args.partition_cache, f"part_n{args.n}_d{args.draws}_s{args.seed}_"
                                                 f"l{args.levels}_{h.hexdigest()[:16]}.npz")
        if os.path.exists(key):
            with np.load(key, allow_pickle=False) as z:
                return [(z[f"ip{l}"], z[f"ix{l}"], int(z[f"rc{l}"][0]), int(z[f"rc{l}"][1]))
                        for l in range(int(z["levels"]))], True
    hier = ge.partition(L, 0.125)[:args.levels]
    if key:
        os.makedirs(args.partition_cache, exist_ok=True)
        arrs = {"levels": np.array(len(hier))}
        for l, (ip, ix, r, c) in enumerate(hier):
            arrs.update({f"ip{l}": ip, f"ix{l}": ix, f"rc{l}": np.array([r, c])})
        np.savez(key + ".tmp.npz", **arrs)
        os.replace(key + ".tmp.npz", key)
    return hier, False


def run_c3(args, rank, world, local, dev):
    """configs[2] (C3): R-MAT 1M draw -> LCC -> partition(A, 0.125), first 4 P_T
    (examples/embedder.cpp:189-192 pattern) -> P^T A P per level on the device.
    One step = one forceAtlasMultilevel call on level 0 (100 iterations,
    src/embed.cpp:793); value = level-0 iterations/s."""
    import torch
    import ge_amd as ge
    t0 = time.perf_counter()
    A = ge.rmat_csr(args.n, args.draws, seed=args.seed)
    L = ge.largest_component(A)
    t_gen = time.perf_counter() - t0
    n0, nnz0 = len(L[0]) - 1, len(L[1])
    t0 = time.perf_counter()
    hier, cached = partition_levels(L, args)
    t_part = time.perf_counter() - t0
    log(rank, f"LCC n={n0} nnz={nnz0} (gen {t_gen:.1f}s), partition {t_part:.1f}s"
              f"{' (cache)' if cached else ''}, levels {[h[2] for h in hier]}")
    ctx = ge.Context(local)
    t0 = time.perf_counter()
    As = [L]
    for PT in hier:
        As.append(ctx.ptap(As[-1], PT))
    t_ptap = time.perf_counter() - t0
    PT = hier[0]
    m = PT[2]
    vA = ge.vertex_of(PT)
    cA = ge.uniform_stream(args.seed + 1, m * args.dim).reshape(m, args.dim)
    rA = 0.01 + 0.19 * (ge.uniform_stream(args.seed + 2, m) + 1.0) / 2.0
    init = ge.uniform_stream(args.seed, n0 * args.dim)  # reference draw order
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d = dict(ip=T(L[0]), ix=T(L[1]), dx=T(L[2]), pip=T(PT[0]), pix=T(PT[1]), vA=T(vA),
             cA=T(cA), rA=T(rA), init=T(init))
    X = torch.zeros((n0, args.dim), dtype=torch.float64, device=dev)
    # a dedicated (non-null) stream made torch's current one: the library launches
    # on it, and torch events and collectives order against it
    work = torch.cuda.Stream(dev)
    torch.cuda.set_stream(work)
    ctx.set_stream(work.cuda_stream)
    torch.cuda.synchronize(dev)  # inputs and X's fill are done before the work stream runs
    # aggregates dealt to ranks by cost (LPT); no collective inside the 100
    # iterations, one member all-gather per call
    from ge_amd.dist import aggregate_cost, assign_aggregates, member_rows, allgather_members
    owned, loads = assign_aggregates(aggregate_cost(PT[0], L[0], PT[1]), world)
    rows = [member_rows(PT[0], PT[1], o) for o in owned]
    log(rank, f"aggregate shards: loads {[f'{x:.3g}' for x in loads]}")
    plan = ge.FamlPlan(ctx, n0, d["ip"].data_ptr(), d["ix"].data_ptr(), d["dx"].data_ptr(),
                       PT[0], d["pip"].data_ptr(), d["pix"].data_ptr(), d["vA"].data_ptr(),
                       args.dim, iterations=args.ml_iterations,
                       aggs=owned[rank] if world > 1 else None)

    def run():
        plan.run(d["cA"].data_ptr(), d["rA"].data_ptr(), d["init"].data_ptr(), X.data_ptr())
        allgather_members(X, rows, rank, world)

    import torch.distributed as dist
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize(dev)
    plan.set_profiling(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.steps):
        run()
    e1.record()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    run_ms = e0.elapsed_time(e1) / args.steps
    res_ms, str_ms, _ = plan.kernel_ms()
    rep_ms, rep_launches, rep_pairs = plan.repulse_ms()
    traffic, traffic_src = pmc_traffic_per_launch("faml_big_repulse", args.workload)
    finite = bool(torch.isfinite(X).all().item())
    sizes = np.diff(PT[0]).astype(np.float64)
    pairs = float((sizes * (sizes - 1)).sum())
    flops = FLOPS_PER_PAIR * pairs * args.ml_iterations
    its = args.steps * args.ml_iterations / elapsed
    tflops = flops / (run_ms * 1e-3) / 1e12  # whole level, all kernels
    rep_flops = FLOPS_PER_PAIR * rep_pairs
    rep_tflops = rep_flops / (rep_ms * 1e-3) / 1e12 if rep_ms > 0 else 0.0
    result = {
        "metric": METRIC, "value": its, "unit": "iterations/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": ("C4 (BASELINE.json configs[3])" if args.workload == "c4" else
                                "C3 (BASELINE.json configs[2])") + ": level-0 forceAtlasMultilevel "
                               f"({args.ml_iterations} iterations per step) on the LCC of a "
                               f"Graph500 R-MAT ({args.n} ids, {args.draws} draws), "
                               "partition(A, 0.125) first 4 levels, strict fp64",
                   "n": n0, "nnz": nnz0, "aggregates": m, "dim": args.dim,
                   "levels": [h[2] for h in hier],
                   "parallelism": f"aggregates{world}" + ("+member-allgather" if world > 1 else "")},
        "edges_per_s": nnz0 * its,
        "pair_interactions_per_s": pairs * its,
        "finite": finite,
        "setup_seconds": {"graph": t_gen, "partition_host": t_part,
                          "partition_from_cache": cached, "ptap_device": t_ptap},
        "roofline": {"kernel": "faml_big_repulse (streamed in-aggregate all-pairs, fp64)",
                     "bound": "mfma", "pipe": "fp64 VALU (dense FP64 peak 78.6 TFLOP/s, spec)",
                     "achieved": rep_tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": rep_tflops / FP64_PEAK_TFLOPS, "traffic": traffic,
                     "traffic_source": traffic_src, "flops_per_launch": rep_flops,
                     "avg_launch_ms": rep_ms, "launches": rep_launches},
        "level_rate": {"flops_per_step": flops, "ms_per_step_device": run_ms,
                       "tflops_all_kernels": tflops, "resident_ms": res_ms,
                       "streamed_ms": str_ms},
    }
    if args.end_to_end:
        t0 = time.perf_counter()
        Xe = ctx.embed(As, hier, args.dim, seed=args.seed)
        result["embed_seconds_end_to_end"] = time.perf_counter() - t0
        result["embed_finite"] = bool(np.isfinite(Xe).all())
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_ml(L, PT, vA, cA, rA, args.dim,
                                                 args.cpu_baseline_seconds, rank)
        result["vs_cpu_baseline"] = its / result["cpu_baseline"]["value"]
    plan.close()
    if args.sweep_slots:  # streamed-path row slots per lane (tuning aid, stderr only)
        for R, U, B in ((1, 1, 8), (1, 1, 5), (1, 1, 4), (1, 1, 3), (1, 2, 4), (2, 1, 4)):
            os.environ["GE_FAML_R"] = str(R)
            os.environ["GE_FAML_U"] = str(U)
            os.environ["GE_FAML_BLOCKS_PER_CU"] = str(B)
            p2 = ge.FamlPlan(ctx, n0, d["ip"].data_ptr(), d["ix"].data_ptr(), d["dx"].data_ptr(),
                             PT[0], d["pip"].data_ptr(), d["pix"].data_ptr(), d["vA"].data_ptr(),
                             args.dim, iterations=args.ml_iterations)
            p2.run(d["cA"].data_ptr(), d["rA"].data_ptr(), d["init"].data_ptr(), X.data_ptr())
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            p2.run(d["cA"].data_ptr(), d["rA"].data_ptr(), d["init"].data_ptr(), X.data_ptr())
            torch.cuda.synchronize(dev)
            log(rank, f"sweep R={R} U={U} blocks/CU={B}: "
                      f"{1e3 * (time.perf_counter() - t0):.1f} ms per call")
            p2.close()
        os.environ.pop("GE_FAML_R")
        os.environ.pop("GE_FAML_U")
        os.environ.pop("GE_FAML_BLOCKS_PER_CU")
    ctx.close()
    if rank == 0:
        print(json.dumps(result), flush=True)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # GE_DIST_BACKEND=gloo rehearses N ranks on one GPU (ranks share cuda:0);
    # the real multi-GPU run is one rank per GPU over RCCL ("nccl")
    backend = os.environ.get("GE_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    if args.workload == "c4":  # configs[3]: 10M ids, 80M draws
        args.n, args.draws = 10_000_000, 80_000_000
    if args.workload in ("c3", "c4"):
        run_c3(args, rank, world, local, dev)
        if world > 1:
            dist.destroy_process_group()
        return

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
    # a dedicated (non-null) stream made torch's current one: the library launches
    # on it, and torch events and collectives order against it
    work = torch.cuda.Stream(dev)
    torch.cuda.set_stream(work)
    ctx.set_stream(work.cuda_stream)
    torch.cuda.synchronize(dev)  # the coordinate upload is done before the work stream runs
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
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
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
    traffic, traffic_src = pmc_traffic_per_launch("fa_repulse", "c2")
    att_traffic, _ = pmc_traffic_per_launch("FaRows", "c2")

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
            "kernel": "tile_rows_kernel<FaRows> + classed_rows_kernel<FaRows> on a side stream "
                      "(CSR attraction + gravity + update; time = both, fork to join)",
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
