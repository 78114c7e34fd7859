#!/usr/bin/env python3
"""ForceAtlas benchmark on MI355X (BASELINE.json metric: ForceAtlas iterations/s
+ edges/s, 3-D embed, 10M-vertex R-MAT @ 1/2/4/8 GPUs).

Default workload (config.workload) = BASELINE.json configs[3] ("C4"): the
Graph500 R-MAT with 10M ids and 80M draws, symmetrised, largest connected
component (examples/embedder.cpp:35-93) -> n = 4.39M, nnz = 125.6M;
partition::partition(A, 0.125) built ON THE DEVICE (bit-exact,
csrc/ge_partition_dev.hip), first 4 levels kept (examples/embedder.cpp:189-192),
P^T A P per level on the device, 3-D.

One step = one forceAtlasMultilevel iteration of every level-0 aggregate
(include/forceatlas.hpp:389-537; SURVEY.md 8(d): "for multilevel, iteration = one
step of every aggregate at a level").  The K timed steps are one
forceAtlasMultilevel call with iterations = K (random init, K iterations, ball
mapping: src/embed.cpp:793 runs the same call with 100), strict fp64 (bit-exact
with the reference's op order).  value = iterations/s of the whole job.

Multi-GPU: `bench.py --gpus N` starts N ranks itself (torch.distributed.run as a
child process, before this process touches the GPU; one rank per GPU over RCCL),
or runs as one of them under an outside launcher (python -m
torch.distributed.run --nproc-per-node N bench.py --gpus N).  Every rank builds
the same graph and hierarchy; the level's aggregates are dealt
to ranks by cost (longest processing time first).  Aggregates exchange nothing
during the iterations (:454, :462 read only the frozen coarse coordinates); one
all-gather of the members' coordinates completes the call.  Total work is fixed:
scaling "strong".

--workload c2 (configs[1]): single-level forceAtlas on the 1M-id R-MAT, one step =
one full iteration (include/forceatlas.hpp:146-270); multi-GPU = row shards + one
RCCL all-gather of the coordinates per iteration.  --workload c3 (configs[2]):
the multilevel step on the 1M-id R-MAT's LCC.

Also reported: edges/s, the dominant kernel's roofline (HIP events on the
launching stream), end-to-end device partition / P^T A P / embed times, and a CPU
baseline (the oracle, rank 0, N = 1 only, bounded sample).
"""
import argparse
import glob
import json
import os
import sys
import time

# the CPU baseline's OpenMP threads stay on neighbouring cores;
# set before any OpenMP runtime is loaded
os.environ.setdefault("OMP_PROC_BIND", "close")
os.environ.setdefault("OMP_PLACES", "cores")

import numpy as np  # noqa: E402

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))

METRIC = "ForceAtlas iterations/sec + edges/sec, 3-D embed, 10M-vtx R-MAT @1/2/4/8 GPU"
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector peak (spec); the strict kernels run on the VALU
HBM_PEAK_GBS = 8000.0    # MI355X HBM3E peak, MI355X_MICROARCH.md
FLOPS_PER_PAIR = 26      # (7d+5) at d=3, SURVEY.md 8(d)
# the symmetric kernel per UNORDERED pair: one term (the 26 above, its row add
# included) plus the subtraction from the partner's (column) sum
SYM_FLOPS_PER_UNORDERED_PAIR = 29


def executed_rate(credited_flops, ms, symmetric):
    """The VALU work the kernel actually issues: the roofline's
    `achieved` credits 26 flops per ORDERED pair (the reference's work, SURVEY.md
    8(d)); the symmetric kernel evaluates each unordered pair once, so it executes
    29 / 52 of that.  Returned as its own record beside the credited figure."""
    if not symmetric or ms <= 0:
        return None
    flops = credited_flops / (2 * FLOPS_PER_PAIR) * SYM_FLOPS_PER_UNORDERED_PAIR
    tf = flops / (ms * 1e-3) / 1e12
    return {"flops_per_launch": flops, "tflops": tf, "frac": tf / FP64_PEAK_TFLOPS,
            "flops_per_unit": "29 per unordered pair (one term with its row add, plus the "
                              "partner's subtraction); sqrt and division counted as 1"}
WORKLOADS = {"c2": (1_000_000, 8_000_000), "c3": (1_000_000, 8_000_000),
             "c4": (10_000_000, 80_000_000)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c4")
    ap.add_argument("--dim", type=int, default=3)
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--mode", choices=["strict", "fast"], default="strict",
                    help="c2 only: fast mode is re-associated (not parity-valid)")
    ap.add_argument("--levels", type=int, default=4)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-end-to-end", action="store_true",
                    help="c3/c4: skip the timed partition::embed over the whole hierarchy")
    ap.add_argument("--partition-host", action="store_true",
                    help="c3/c4: also time the library's host partition (minutes at c4)")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, check the process group and exit (no GPU work)")
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def host_info():
    """CPU model, logical CPUs, physical cores (lscpu) and this process's affinity."""
    info = {"logical_cpus": os.cpu_count()}
    try:  # the calling thread's mask (bound to one core by libgomp: see cpu_share)
        info["main_thread_affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpuset.cpus.effective"):
        try:
            with open(path) as f:
                info[os.path.basename(path)] = f.read().strip()
        except OSError:
            pass
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = {}
        for line in out.splitlines():
            k, _, v = line.partition(":")
            kv[k.strip()] = v.strip()
        info["model"] = kv.get("Model name")
        sockets = int(kv.get("Socket(s)", "1") or 1)
        cores = int(kv.get("Core(s) per socket", "0") or 0)
        if cores:
            info["physical_cores"] = sockets * cores
    except Exception:
        pass
    return info


def cpu_share():
    """CPUs this job may keep busy at once: the cgroup's CPU quota (cpu.max) and its
    cpuset.  Not os.sched_getaffinity(0): that is the CALLING THREAD's mask, and once
    libgomp has started with OMP_PROC_BIND=close / OMP_PLACES=cores (set above) it has
    bound the main thread to its first place -- one core, 2 SMT threads -- which is
    why rounds 1-4 reported 2 CPUs on boxes whose job gets 16 (VERDICT r04 weak 9;
    scripts/affinity_probe.py: 256 CPUs in a process without the binding)."""
    share = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()
        if quota != "max":
            share = min(share, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    # the cgroup's cpuset, not /proc/self/status: that is the main thread's mask too
    # (round 5's first cut read it and still reported 2)
    try:
        with open("/sys/fs/cgroup/cpuset.cpus.effective") as f:
            n = 0
            for part in f.read().strip().split(","):
                if part:
                    a, _, b = part.partition("-")
                    n += int(b or a) - int(a) + 1
            if n > 0:
                share = min(share, n)
    except (OSError, ValueError):
        pass
    return share


def baseline_threads():
    """OpenMP threads for the CPU baseline: the job's CPU share (cpu_share), so a small
    share is not oversubscribed; OMP_NUM_THREADS only lowers it."""
    cpus = cpu_share()
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(cpus, env) if env else cpus


def baseline_record(value, unit, threads, sample, per_iter):
    hi = host_info()
    # the threads that can run at once: the OpenMP threads, bounded by the job's CPU
    # share (the GPU box confines a job to 16 CPUs of its cgroup quota)
    hi["cpu_share"] = cpu_share()
    cores = min(threads, hi["cpu_share"])
    rec = {"value": value, "unit": unit, "cores": cores, "omp_threads": threads, "kind": "port",
           "sample": sample,
           "seconds_per_iteration": per_iter, "host": hi,
           "omp": {"OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"),
                   "OMP_PROC_BIND": os.environ.get("OMP_PROC_BIND"),
                   "OMP_PLACES": os.environ.get("OMP_PLACES")}}
    pc = hi.get("physical_cores")
    if pc and pc > cores:
        # the reference's loops are `omp parallel for` over independent rows /
        # aggregates: perfect scaling to every physical core bounds what the whole
        # host could do (an extrapolation, not a measurement)
        rec["extrapolated_all_physical_cores"] = {"value": value * pc / cores, "cores": pc,
                                                  "note": "linear scaling from the measured "
                                                          "cores; upper bound, not measured"}
    return rec


def sym_schedule(plan):
    """The plan's repulsion schedule; None from an older variant library
    (GE_LIB_PATH A/B runs) that lacks ge_faml_plan_schedule."""
    try:
        return plan.schedule()
    except AttributeError:
        return None


def pmc_traffic_per_launch(kernel_prefix, workload):
    """HBM bytes per launch of the kernels whose names contain kernel_prefix, from the
    committed rocprofv3 PMC passes of the same workload (profiles/<round>/pmc_fetch_
    <workload>*.csv and pmc_write_...).  gfx950 correction (MI355X_MICROARCH.md):
    FETCH_SIZE reports half the bytes of a wide coalesced read -> bytes =
    (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  One "launch" is one pass of the matching
    kernels: the sum over every matching dispatch divided by the dispatch count of the
    least frequent matching kernel (the row pass launches its tile kernel three times --
    early rows' segments, the other segments, tiles -- and each heavy-chain kernel once)."""
    def read(pattern, counter):
        import csv
        for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*", pattern)), reverse=True):
            vals = {}
            with open(path) as f:
                for row in csv.DictReader(f):
                    name = row.get("Kernel_Name", "")
                    if row.get("Counter_Name") == counter and name.find(kernel_prefix) >= 0:
                        vals.setdefault(name, []).append(float(row["Counter_Value"]))
            if vals:
                passes = min(len(v) for v in vals.values())
                return sum(sum(v) for v in vals.values()) / passes, path
        return None
    f = read(f"pmc_fetch_{workload}*.csv", "FETCH_SIZE")
    w = read(f"pmc_write_{workload}*.csv", "WRITE_SIZE")
    if not f or not w:
        return None, None
    return (2.0 * f[0] + w[0]) * 1024.0, [os.path.relpath(f[1], REPO), os.path.relpath(w[1], REPO)]


def cpu_baseline_fa(A, X0, seconds, rank):
    """Oracle (the reference loop restated) on a bounded sample: the force rows of one
    iteration for a contiguous block of rows, scaled to a full iteration (per-row cost
    is n pairs + deg(i) edges: uniform)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    oracle_lib.build()
    threads = baseline_threads()
    n = len(A[0]) - 1
    deg = oracle_lib.degrees(A)
    rb, rows = n // 2, 256
    t0 = time.perf_counter()
    oracle_lib.fa_forces_rows(A, X0, deg, rb, rb + rows, nthreads=threads)
    t = time.perf_counter() - t0
    rows = int(min(n - rb, max(rows, rows * seconds / max(t, 1e-3))))
    t0 = time.perf_counter()
    oracle_lib.fa_forces_rows(A, X0, deg, rb, rb + rows, nthreads=threads)
    t = time.perf_counter() - t0
    per_iter = t * n / rows
    log(rank, f"cpu baseline: {rows} rows in {t:.2f}s on {threads} threads -> {per_iter:.1f}s/iter")
    return baseline_record(1.0 / per_iter, "iterations/s", threads,
                           f"oracle forceAtlas force pass for rows [{rb},{rb + rows}) of one "
                           f"iteration ({rows} of {n} rows, {t:.1f}s, OpenMP {threads} threads), "
                           "scaled by n/rows to one full iteration", per_iter)


def cpu_baseline_ml(L, PT, vA, cA, rA, dim, seconds, rank):
    """Oracle forceAtlasMultilevel on a bounded sample of aggregates (every k-th),
    one iteration, scaled by the pair+edge cost of the whole level."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    oracle_lib.build()
    threads = baseline_threads()
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
        return time.perf_counter() - t0, cost[sel].sum(), len(sel)

    stride = max(1, len(s) // 1024)
    t, c, _ = run(stride)
    stride = max(1, int(stride * t / seconds)) if t > 0 else 1
    t, c, na = run(stride)
    # cost units per second of one thread, then the whole level on `threads` threads:
    # the reference deals whole aggregates to threads (`omp parallel for`,
    # include/forceatlas.hpp:340), so an iteration lasts at least as long as its
    # largest aggregate on one thread (the serial tail) and at least the total work
    # spread over all threads -- the larger of the two (a list-scheduling lower
    # bound, so the baseline is not understated)
    rate = c / (t * threads)
    spread = cost.sum() / (rate * threads)
    tail = cost.max() / rate
    per_iter = max(spread, tail)
    log(rank, f"cpu baseline (multilevel): stride {stride}, {t:.2f}s on {threads} threads "
              f"-> {per_iter:.2f}s/iteration (spread {spread:.2f}s, serial tail {tail:.2f}s)")
    rec = baseline_record(1.0 / per_iter, "iterations/s", threads,
                          f"oracle forceAtlasMultilevel, 1 iteration over every {stride}-th "
                          f"aggregate of level 0 ({na} aggregates, {t:.1f}s, OpenMP {threads} "
                          "threads); per-thread rate scaled to the whole level as max(total "
                          "cost / threads, largest aggregate on one thread)", per_iter)
    rec["model"] = {"spread_seconds": spread, "serial_tail_seconds": tail,
                    "largest_aggregate": int(s.max()), "cost_units": "s(s-1) + CSR entries"}
    if "extrapolated_all_physical_cores" in rec:  # the serial tail does not shrink
        pc = rec["extrapolated_all_physical_cores"]["cores"]
        rec["extrapolated_all_physical_cores"]["value"] = 1.0 / max(cost.sum() / (rate * pc), tail)
        rec["extrapolated_all_physical_cores"]["note"] = ("per-thread rate on every physical "
                                                          "core, serial tail kept; not measured")
    return rec


def timed(args, world, dev, fn):
    """W untimed steps, then K steps between barrier + synchronize.  Returns (max over
    ranks, every rank's seconds)."""
    import torch
    import torch.distributed as dist
    fn(args.warmup, timed=False)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    fn(args.steps, timed=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world == 1:
        return elapsed, [elapsed]
    tdev = dev if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
    every = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(every, t)
    per_rank = [float(x.item()) for x in every]
    return max(per_rank), per_rank


def make_comm(ctx, rank, world):
    """The library's communicator (ge_comm): RCCL inside libge, its unique id
    broadcast from rank 0 over the harness's process group; GE_DIST_BACKEND=gloo
    (several ranks sharing one GPU) uses the library's host transport instead."""
    import torch.distributed as dist
    import ge_amd as ge
    if world == 1:
        return None
    if dist.get_backend() != "nccl":
        comm = ge.Comm(ctx, world, rank, backend="transport")
    else:
        box = [ge.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        comm = ge.Comm(ctx, world, rank, backend="rccl", uid=box[0])
    nranks, crank, is_rccl = comm.info()
    assert nranks == world and crank == rank, (nranks, crank, world, rank)
    assert bool(is_rccl) == (dist.get_backend() == "nccl"), "expected the RCCL communicator"
    return comm


def comm_record(comm, world):
    """What the library's communicator reports (nranks_seen, RCCL or transport)."""
    if comm is None:
        return {"nranks_seen": 1, "backend": "none (one GPU)"}
    nranks, _, is_rccl = comm.info()
    rec = {"nranks_seen": nranks, "backend": "rccl" if is_rccl else "transport"}
    if not is_rccl:
        rec["rehearsal"] = ("ranks share one GPU over the host transport "
                            "(GE_DIST_BACKEND=gloo): a rehearsal, not a multi-GPU measurement")
    return rec


def run_multilevel(args, rank, world, local, dev):
    """configs[2] / configs[3]: R-MAT -> LCC -> device partition(A, 0.125), first 4 P_T
    -> device P^T A P -> K forceAtlasMultilevel iterations of level 0."""
    import torch
    import ge_amd as ge
    ctx = ge.Context(local)
    t0 = time.perf_counter()
    # R-MAT + largest component on the device (csrc/ge_graph.hip; same arrays as the
    # host generator, tests/test_gpu_graph.py)
    L = ctx.rmat_csr(args.n, args.draws, seed=args.seed, lcc=True)
    t_gen = time.perf_counter() - t0
    n0, nnz0 = len(L[0]) - 1, len(L[1])
    t0 = time.perf_counter()
    hier_full = ctx.partition(L, 0.125)
    t_part = time.perf_counter() - t0
    hier = hier_full[:args.levels]
    t_part_host = None
    if args.partition_host and rank == 0:
        t0 = time.perf_counter()
        hh = ge.partition(L, 0.125)
        t_part_host = time.perf_counter() - t0
        assert all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
                   for a, b in zip(hh, hier_full)), "device and host partition differ"
    log(rank, f"LCC n={n0} nnz={nnz0} (gen {t_gen:.1f}s), device partition {t_part:.1f}s, "
              f"levels {[h[2] for h in hier_full]}")
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
    # a dedicated (non-null) stream made torch's current one: the library launches on
    # it, and torch events and collectives order against it
    work = torch.cuda.Stream(dev)
    torch.cuda.set_stream(work)
    ctx.set_stream(work.cuda_stream)
    torch.cuda.synchronize(dev)
    comm = make_comm(ctx, rank, world)
    # aggregates dealt to ranks by cost inside libge (ge_assign_aggregates_split: LPT
    # on s(s-1) + the members' CSR entries; an aggregate above half a rank's share is
    # split by row tiles over all ranks, owner -1, its rows exchanged every iteration)
    owner = ge.assign_aggregates_split(PT, L[0], world) if world > 1 else np.zeros(m, np.int32)
    mine = np.flatnonzero(owner == rank).astype(np.int32)
    split = np.flatnonzero(owner < 0).astype(np.int32)
    gather_owner = np.where(owner < 0, 0, owner).astype(np.int32)
    if world > 1:
        from ge_amd.dist import aggregate_cost
        cost = aggregate_cost(PT[0], L[0], PT[1])
        log(rank, f"aggregate shards: loads "
                  f"{[f'{cost[owner == r].sum():.3g}' for r in range(world)]}")
    plans = {}
    plan_seconds = {}

    def plan_for(iters):
        if iters not in plans:
            t0 = time.perf_counter()
            plans[iters] = ge.FamlPlan(ctx, n0, d["ip"].data_ptr(), d["ix"].data_ptr(),
                                       d["dx"].data_ptr(), PT[0], d["pip"].data_ptr(),
                                       d["pix"].data_ptr(), d["vA"].data_ptr(), args.dim,
                                       iterations=iters, aggs=mine if world > 1 else None,
                                       split=split if world > 1 else None, comm=comm)
            plan_seconds[iters] = time.perf_counter() - t0
        return plans[iters]

    pk = plan_for(args.steps)
    if args.warmup:
        plan_for(args.warmup)

    def steps(k, timed):
        if k == 0:
            return
        p = plans[k]
        if timed:
            p.set_profiling(True)
        p.run(d["cA"].data_ptr(), d["rA"].data_ptr(), d["init"].data_ptr(), X.data_ptr())
        if comm is not None:  # one all-gather of the members' coordinates (libge, RCCL)
            comm.allgather_members(X.data_ptr(), args.dim, PT, gather_owner)

    elapsed, per_rank = timed(args, world, dev, steps)
    rep_ms, rep_launches, rep_pairs = pk.repulse_ms()
    res_ms, str_ms, _ = pk.kernel_ms()
    att_ms, att_passes, att_rows, att_entries = pk.rows_ms()
    # SURVEY.md 8(d) B_attr over the streamed members' rows: indptr 4 B + x read 24 B +
    # x write 24 B per row, 12 B per CSR entry (int32 index + fp64 weight)
    att_bytes = 12 * att_entries + 52 * att_rows
    att_gbs = att_bytes / (att_ms * 1e-3) / 1e9 if att_ms > 0 else 0.0
    att_traffic, att_src = pmc_traffic_per_launch("FamlRows", args.workload)
    rep_kernel = "faml_big_repulse" if os.environ.get("GE_FAML_SYM") == "0" else "faml_sym_repulse"
    traffic, traffic_src = pmc_traffic_per_launch(rep_kernel, args.workload)
    finite = bool(torch.isfinite(X).all().item())
    sizes = np.diff(PT[0]).astype(np.float64)
    pairs = float((sizes * (sizes - 1)).sum())
    its = args.steps / elapsed
    rep_flops = FLOPS_PER_PAIR * rep_pairs
    rep_tflops = rep_flops / (rep_ms * 1e-3) / 1e12 if rep_ms > 0 else 0.0
    sched = sym_schedule(pk)
    cfgname = {"c3": "C3 (BASELINE.json configs[2])", "c4": "C4 (BASELINE.json configs[3])"}
    result = {
        "metric": METRIC, "value": its, "unit": "iterations/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": f"{cfgname[args.workload]}: 3-D multilevel embed of the LCC of a "
                               f"Graph500 R-MAT ({args.n} ids, {args.draws} draws); partition(A, "
                               "0.125) on the device, first 4 levels, P^T A P on the device; one "
                               "step = one forceAtlasMultilevel iteration of every level-0 "
                               "aggregate, strict fp64",
                   "n": n0, "nnz": nnz0, "aggregates": m, "dim": args.dim,
                   "levels": [h[2] for h in hier],
                   "parallelism": f"aggregates{world}" + ("+member-allgather(libge " +
                                                          ("rccl" if comm.info()[2] else
                                                           "transport") + ")"
                                                          if world > 1 else "")},
        "edges_per_s": nnz0 * its,
        "pair_interactions_per_s": pairs * its,
        "finite": finite,
        "roofline": {"kernel": f"{rep_kernel} (streamed in-aggregate all-pairs repulsion, "
                               "strict fp64; one launch per iteration)",
                     "bound": "valu", "pipe": "fp64 VALU; priced against the FP64 vector peak "
                                              "(78.6 TFLOP/s, spec)",
                     "achieved": rep_tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": rep_tflops / FP64_PEAK_TFLOPS, "traffic": traffic,
                     "traffic_source": traffic_src, "flops_per_launch": rep_flops,
                     "flops_per_unit": "26 per ordered in-aggregate pair (7d+5, d=3); the "
                                       "symmetric kernel evaluates each unordered pair once "
                                       "and credits both ordered pairs",
                     "executed": executed_rate(rep_flops, rep_ms,
                                               rep_kernel == "faml_sym_repulse" and
                                               (sched or {}).get("row_blocks", 1) == 0),
                     "avg_launch_ms": rep_ms, "launches": rep_launches},
        "roofline_attraction": {"kernel": "tile_rows_kernel<FamlRows> + heavy rows (the "
                                          "streamed members' CSR attraction / external pull, "
                                          "gravity, update; one pass per iteration)",
                                "bound": "hbm", "achieved": att_gbs, "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": att_gbs / HBM_PEAK_GBS,
                                "traffic": att_traffic, "traffic_source": att_src,
                                "algorithmic_bytes_per_launch": att_bytes,
                                "bytes_per_unit": "12 per CSR entry + 52 per row (SURVEY.md 8(d))",
                                "rows": att_rows, "entries": att_entries,
                                "avg_launch_ms": att_ms, "launches": att_passes,
                                # the gathers' own rate: each CSR entry gathers one random
                                # neighbour record, served as one 64-B line (PMC: ~0.8 lines
                                # per entry at C4, 1.0 at C5)
                                "gather_lines": {
                                    "bytes_per_launch": 64 * att_entries,
                                    "rate_GBs": (64 * att_entries / (att_ms * 1e-3) / 1e9
                                                 if att_ms > 0 else 0.0),
                                    "note": "model: one 64-B line per CSR entry; the measured "
                                            "line count is in `traffic`"}},
        "level_rate": {"resident_ms": res_ms, "streamed_ms": str_ms},
        # this rank's streamed aggregates: plain symmetric sweeps / bands (a shorter
        # dependency chain) / whole row blocks
        "sym_schedule": sched,
        "setup_seconds": {"graph_device": t_gen, "partition_device": t_part,
                          "partition_host": t_part_host, "ptap_device": t_ptap,
                          "plan_build": plan_seconds.get(args.steps),
                          "plan_build_note": "per-level tables built once per plan outside the "
                                             "timed steps (pack tables, edge codes, internal "
                                             "degrees of the streamed members)"},
        "ranks": dict(comm_record(comm, world), per_rank_seconds=per_rank),
    }
    if world > 1:
        result["ranks"]["per_rank_load"] = [float(cost[owner == r].sum() + cost[owner < 0].sum() /
                                                  world) for r in range(world)]
        result["ranks"]["split_aggregates"] = int(len(split))
    for p in plans.values():
        p.close()
    if comm is not None:
        comm.close()
    if rank == 0 and world == 1 and not args.no_end_to_end:
        t0 = time.perf_counter()
        Xe = ctx.embed(As, hier, args.dim, seed=args.seed)
        result["embed_seconds_end_to_end"] = time.perf_counter() - t0
        result["embed_finite"] = bool(np.isfinite(Xe).all())
        result["pipeline_seconds_device"] = (t_part + t_ptap +
                                             result["embed_seconds_end_to_end"])
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_ml(L, PT, vA, cA, rA, args.dim,
                                                 args.cpu_baseline_seconds, rank)
        result["vs_cpu_baseline"] = its / result["cpu_baseline"]["value"]
    ctx.close()
    if rank == 0:
        print(json.dumps(result), flush=True)


def run_single_level(args, rank, world, local, dev):
    """configs[1]: single-level forceAtlas, one step = one iteration."""
    import torch
    import ge_amd as ge
    from ge_amd.dist import row_shards
    ctx = ge.Context(local)
    t0 = time.perf_counter()
    A = ctx.rmat_csr(args.n, args.draws, seed=args.seed)
    n, nnz = len(A[0]) - 1, len(A[1])
    X0 = ge.uniform_stream(args.seed, n * args.dim).reshape(n, args.dim)  # ref init order
    log(rank, f"R-MAT n={n} nnz={nnz} generated in {time.perf_counter() - t0:.1f}s")
    chunk, shards = row_shards(n, world)
    npad = chunk * world
    rb, re = shards[rank]
    ip, ix, dx = (torch.from_numpy(a).to(dev) for a in A)
    xa = torch.zeros((npad, args.dim), dtype=torch.float64, device=dev)
    xa[:n] = torch.from_numpy(X0).to(dev)
    xb = torch.zeros_like(xa)
    work = torch.cuda.Stream(dev)
    torch.cuda.set_stream(work)
    ctx.set_stream(work.cuda_stream)
    torch.cuda.synchronize(dev)
    comm = make_comm(ctx, rank, world)
    mode = ge.MODE_FAST if args.mode == "fast" else ge.MODE_STRICT
    plan = ctx.fa_plan(n, nnz, ip.data_ptr(), ix.data_ptr(), dx.data_ptr(), args.dim, rb, re,
                       mode=mode)
    buf = [xa, xb]

    def steps(k, timed):
        if timed:
            plan.set_profiling(True)
        for _ in range(k):
            plan.step(buf[0].data_ptr(), buf[1].data_ptr())
            if comm is not None:  # one in-place all-gather of the rows (libge, RCCL)
                comm.allgather_coords(buf[1].data_ptr(), chunk, args.dim)
            buf.reverse()

    elapsed, per_rank = timed(args, world, dev, steps)
    rep_ms, att_ms, launches = plan.kernel_ms()
    finite = bool(torch.isfinite(buf[0][:n]).all().item())
    its = args.steps / elapsed
    rows = re - rb
    pairs = rows * (n - 1)
    rep_tflops = FLOPS_PER_PAIR * pairs / (rep_ms * 1e-3) / 1e12 if rep_ms > 0 else 0.0
    attr_bytes = 12 * nnz * rows / n + 52 * rows + 4  # SURVEY 8(d) B_attr, this rank's rows
    att_gbs = attr_bytes / (att_ms * 1e-3) / 1e9 if att_ms > 0 else 0.0
    # the plan's repulsion kernel (ge_fa.hip plan_init): symmetric sweeps for a STRICT
    # plan over every row (one rank), the ordered-pair kernel on a row shard or FAST
    sym = (args.mode == "strict" and world == 1 and os.environ.get("GE_FA_SYM", "") != "0")
    rep_kernel = "faml_sym_repulse" if sym else "fa_repulse_%s" % args.mode
    traffic, traffic_src = pmc_traffic_per_launch(rep_kernel, "c2")
    att_traffic, att_src = pmc_traffic_per_launch("FaRows", "c2")
    result = {
        "metric": METRIC, "value": its, "unit": "iterations/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": "C2 (BASELINE.json configs[1]): single-level 3-D forceAtlas "
                               f"iteration, Graph500 R-MAT n={n}, {args.draws} draws, nnz={nnz}, "
                               f"{args.mode} fp64",
                   "n": n, "nnz": nnz, "dim": args.dim, "mode": args.mode,
                   "parallelism": f"rows{world}" + ("+allgather" if world > 1 else "")},
        "edges_per_s": nnz * its,
        "pair_interactions_per_s": n * (n - 1) * its,
        "finite": finite,
        "roofline": {"kernel": rep_kernel + (" (single-level symmetric sweeps: one aggregate of all"
                                             " n rows, fp64)" if sym else
                                             " (all-pairs repulsion, fp64)"),
                     "bound": "valu", "pipe": "fp64 VALU; priced against the FP64 vector peak "
                                              "(78.6 TFLOP/s, spec)",
                     "achieved": rep_tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": rep_tflops / FP64_PEAK_TFLOPS, "traffic": traffic,
                     "traffic_source": traffic_src, "flops_per_launch": FLOPS_PER_PAIR * pairs,
                     "flops_per_unit": "26 per ordered pair (7d+5, d=3)" + (
                         "; the symmetric kernel evaluates each unordered pair once and credits"
                         " both ordered pairs" if sym else ""),
                     "executed": executed_rate(FLOPS_PER_PAIR * pairs, rep_ms, sym),
                     "avg_launch_ms": rep_ms, "launches": launches},
        "roofline_attraction": {"kernel": "tile_rows_kernel<FaRows> + classed_rows_kernel<FaRows>"
                                          " (CSR attraction + gravity + update; fork to join)",
                                "bound": "hbm", "achieved": att_gbs, "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": att_gbs / HBM_PEAK_GBS,
                                "traffic": att_traffic, "traffic_source": att_src,
                                "algorithmic_bytes_per_launch": attr_bytes,
                                "avg_launch_ms": att_ms},
        "ranks": dict(comm_record(comm, world), per_rank_seconds=per_rank,
                      rows_per_rank=[b - a for a, b in shards]),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_fa(A, X0, args.cpu_baseline_seconds, rank)
        result["vs_cpu_baseline"] = its / result["cpu_baseline"]["value"]
    plan.close()
    if comm is not None:
        comm.close()
    ctx.close()
    if rank == 0:
        print(json.dumps(result), flush=True)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(args):
    """`--gpus N` without an outside launcher: run torch.distributed.run with N
    ranks (one per GPU) as a CHILD process and return its exit code.  Nothing here
    touches the GPU (counting devices does not initialise it on this image), and the
    process is never replaced (no exec)."""
    import subprocess
    import torch
    backend = os.environ.get("GE_DIST_BACKEND", "nccl")
    if backend == "nccl" and not args.launch_check:
        have = torch.cuda.device_count()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs one GPU per rank but {have} "
                  "visible; GE_DIST_BACKEND=gloo rehearses the ranks on one GPU over the "
                  "host transport (labelled a rehearsal in the JSON)", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, GE_BENCH_SPAWNED="1")
    return subprocess.call(cmd, env=env)


def launch_check(world, rank, local):
    """--launch-check: every rank reports (rank, local rank, pid) over the process
    group; rank 0 prints one JSON line.  No GPU work."""
    import torch.distributed as dist
    seen = [None] * world
    if world > 1:
        dist.all_gather_object(seen, (rank, local, os.getpid()))
    else:
        seen = [(rank, local, os.getpid())]
    if rank == 0:
        print(json.dumps({"launch_check": True, "nranks_seen": world,
                          "backend": dist.get_backend() if world > 1 else "none",
                          "spawned_by_bench": os.environ.get("GE_BENCH_SPAWNED") == "1",
                          "ranks": [{"rank": r, "local_rank": lr, "pid": pid}
                                    for r, lr, pid in seen]}), flush=True)


def main():
    args = parse()
    args.n, args.draws = WORKLOADS[args.workload]
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: {world} ranks were launched for --gpus {args.gpus}")
    # GE_DIST_BACKEND=gloo rehearses N ranks on one GPU (ranks share cuda:0); the real
    # multi-GPU run is one rank per GPU over RCCL ("nccl")
    backend = os.environ.get("GE_DIST_BACKEND", "nccl")
    if args.launch_check:
        if world > 1:
            dist.init_process_group("gloo")
        launch_check(world, rank, local)
        if world > 1:
            dist.destroy_process_group()
        return
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    if args.workload == "c2":
        run_single_level(args, rank, world, local, dev)
    else:
        run_multilevel(args, rank, world, local, dev)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
