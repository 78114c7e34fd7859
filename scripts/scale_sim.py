"""Multi-GPU rehearsal on one GPU for the C4 multilevel level: for N = 1, 2, 4, 8
every rank's share (ge_assign_aggregates, the deal bench.py uses) runs as its own
subset plan, one after another, and its kernel time per iteration is measured.
max over ranks approximates the N-GPU step (the member all-gather, once per call,
is left out); efficiency = t(1) / (N * max).  Prints one JSON line per N.

SPLIT_MIN=k (SURVEY.md 8(e) split): aggregates of >= k members are split by row
tiles over all N ranks (ge_assign_aggregates_split), each rank's shard plan runs its
row tiles of them as row blocks and exchanges the split rows after every iteration.
The exchange goes through a local transport that copies the rank's own block into
every slot (finite coordinates, host round trip), so the per-iteration wall time
includes a PCIe copy RCCL would not make; the kernel times (repulse_ms, rows_ms)
are unaffected, and the exchange is priced from its bytes at XGMI_GBS (bus
bandwidth of an RCCL all-gather, default 300 GB/s).

WORKLOAD=c2 (configs[1]): the single-level forceAtlas on the
1M-id R-MAT sharded by rows as bench.py --workload c2 --gpus N does it
(ge_amd.dist.row_shards: contiguous vertex rows per rank, every rank's rows against
all coordinates, one in-place all-gather of the coordinate array per iteration).
Every rank's row-shard plan is timed on this GPU one after another (ITERS steps after
one warm-up step); the all-gather of n * d * 8 bytes is priced at XGMI_GBS.  N = 1
is the whole level (the symmetric sweeps); a shard runs the ordered-pair kernel."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))
import ge_amd as ge  # noqa: E402


def local_comm(ctx, N, r):
    """A ge_comm of N ranks whose all-gather copies this rank's block into every slot."""
    c = ge.Comm.__new__(ge.Comm)
    c.ctx, c.nranks, c.rank = ctx, N, r

    def cb(user, send, recv, nbytes):
        for k in range(N):
            ctypes.memmove(recv + k * nbytes, send, nbytes)
        return 0
    c._cb = ge._ALLGATHER_FN(cb)
    c._tp = ge._Transport(None, c._cb)
    h = ctypes.c_void_p()
    ge._check(ge.lib().ge_comm_create_transport(ctx.h, N, r, ctypes.cast(ctypes.byref(c._tp),
                                                                         ctypes.c_void_p),
                                                ctypes.byref(h)))
    c.h = h
    return c


def main_c2():
    from ge_amd.dist import row_shards
    dim, iters = 3, int(os.environ.get("ITERS", "2"))
    ctx = ge.Context(0)
    A = ctx.rmat_csr(1_000_000, 8_000_000, seed=12345)
    n, nnz = len(A[0]) - 1, len(A[1])
    dev = torch.device("cuda:0")
    ip, ix, dx = (torch.from_numpy(a).to(dev) for a in A)
    X0 = torch.from_numpy(ge.uniform_stream(12345, n * dim).reshape(n, dim)).to(dev)
    gbs = float(os.environ.get("XGMI_GBS", "300"))
    t1 = None
    for N in [int(x) for x in os.environ.get("NS", "1,2,4,8").split(",")]:
        chunk, shards = row_shards(n, N)
        xa = torch.zeros((chunk * N, dim), dtype=torch.float64, device=dev)
        xa[:n] = X0
        xb = torch.zeros_like(xa)
        times, reps, atts = [], [], []
        for r in range(N):
            rb, re = shards[r]
            p = ctx.fa_plan(n, nnz, ip.data_ptr(), ix.data_ptr(), dx.data_ptr(), dim, rb, re)
            p.step(xa.data_ptr(), xb.data_ptr())  # warm-up (the symmetric plan's first launch)
            ctx.sync()
            p.set_profiling(True)
            t0 = time.perf_counter()
            for _ in range(iters):
                p.step(xa.data_ptr(), xb.data_ptr())
            ctx.sync()
            times.append((time.perf_counter() - t0) / iters * 1e3)
            rep_ms, att_ms, _ = p.kernel_ms()
            reps.append(rep_ms)
            atts.append(att_ms)
            p.close()
            print(f"N={N} rank {r}: rows [{rb}, {re}) {times[-1]:.1f} ms per step", file=sys.stderr,
                  flush=True)
        xbytes = n * dim * 8
        ag_ms = xbytes * (N - 1) / N / (gbs * 1e9) * 1e3 if N > 1 else 0.0
        step = max(times) + ag_ms
        t1 = t1 or step
        print(json.dumps({"workload": "c2", "N": N, "ms_per_step_by_rank": times,
                          "repulse_ms_by_rank": reps, "attract_ms_by_rank": atts,
                          "allgather_bytes": xbytes if N > 1 else 0,
                          "allgather_ms_priced": ag_ms, "max_ms": step,
                          "efficiency": t1 / (N * step),
                          "kernel": "symmetric sweeps" if N == 1 else "ordered-pair row shards"}),
              flush=True)
    ctx.close()


def main():
    if os.environ.get("WORKLOAD") == "c2":
        return main_c2()
    n, draws, dim, iters = 10_000_000, 80_000_000, 3, int(os.environ.get("ITERS", "5"))
    ctx = ge.Context(0)
    L = ctx.rmat_csr(n, draws, seed=12345, lcc=True)
    PT = ctx.partition(L, 0.125)[0]
    m = PT[2]
    n0 = len(L[0]) - 1
    vA = ge.vertex_of(PT)
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d = dict(ip=T(L[0]), ix=T(L[1]), dx=T(L[2]), pip=T(PT[0]), pix=T(PT[1]), vA=T(vA),
             cA=T(ge.uniform_stream(7, m * dim)), rA=T(0.01 + 0.19 * (ge.uniform_stream(8, m) + 1) / 2),
             init=T(ge.uniform_stream(5, n0 * dim)))
    X = torch.zeros((n0, dim), dtype=torch.float64, device=dev)
    if os.environ.get("SAVE_LEVEL"):  # level-0 sizes + members' CSR entries, for offline models
        deg = np.diff(L[0]).astype(np.int64)
        ent = np.add.reduceat(deg[PT[1]], PT[0][:-1])
        np.savez(os.environ["SAVE_LEVEL"], pt_ip=PT[0], entries=ent)
    t1 = None
    for N in [int(x) for x in os.environ.get("NS", "1,2,4,8").split(",")]:
        split_min = int(os.environ.get("SPLIT_MIN", "0"))
        if split_min > 0 and N > 1:
            owner = ge.assign_aggregates_split(PT, L[0], N, split_min)
        else:
            owner = ge.assign_aggregates(PT, L[0], N)
        split = np.flatnonzero(owner < 0).astype(np.int32)
        split_rows = int(sum(PT[0][a + 1] - PT[0][a] for a in split))
        times, reps, rows_ms, scheds = [], [], [], []
        for r in range(N):
            mine = np.flatnonzero(owner == r).astype(np.int32)
            # STAMP_N=N: the per-unit timeline of rank 0's last launch (GE_SYM_STAMPS,
            # scripts/sym_timeline.py) into gpurun_out/stamps_N<N>.bin
            if os.environ.get("STAMP_N") == str(N) and r == 0:
                os.environ["GE_SYM_STAMPS"] = os.path.join(REPO, "gpurun_out", f"stamps_N{N}.bin")
            else:
                os.environ.pop("GE_SYM_STAMPS", None)
            comm = local_comm(ctx, N, r) if len(split) else None
            p = ge.FamlPlan(ctx, n0, d["ip"].data_ptr(), d["ix"].data_ptr(), d["dx"].data_ptr(),
                            PT[0], d["pip"].data_ptr(), d["pix"].data_ptr(), d["vA"].data_ptr(),
                            dim, iterations=iters, aggs=mine if N > 1 else None,
                            split=split if comm else None, comm=comm)
            p.run(d["cA"].data_ptr(), d["rA"].data_ptr(), d["init"].data_ptr(), X.data_ptr())
            ctx.sync()
            p.set_profiling(True)
            t0 = time.perf_counter()
            p.run(d["cA"].data_ptr(), d["rA"].data_ptr(), d["init"].data_ptr(), X.data_ptr())
            ctx.sync()
            times.append((time.perf_counter() - t0) / iters * 1e3)
            rep_ms, _, _ = p.repulse_ms()
            reps.append(rep_ms)
            rows_ms.append(p.rows_ms()[0])
            scheds.append(p.schedule())
            p.close()
            if comm:
                comm.close()
        t1 = t1 or times[0]
        rec = {"N": N, "ms_per_iteration_by_rank": times, "max_ms": max(times),
               "repulse_ms_by_rank": reps, "rows_ms_by_rank": rows_ms,
               "schedule_by_rank": scheds, "efficiency": t1 / (N * max(times))}
        if len(split):
            gbs = float(os.environ.get("XGMI_GBS", "300"))
            xbytes = split_rows * dim * 8
            rec.update(split_aggregates=int(len(split)), split_rows=split_rows,
                       exchange_bytes_per_iteration=xbytes,
                       exchange_ms_priced=xbytes * (N - 1) / N / (gbs * 1e9) * 1e3,
                       note="ms_per_iteration includes a host round trip of the exchange")
        print(json.dumps(rec), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
