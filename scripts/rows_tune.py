"""Time the C2 attraction pass (classed_rows_kernel<FaRows>) per degree-class
bounds (GE_ROWS_MED / GE_ROWS_HEAVY), on the 1M R-MAT and on a hub-free graph."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "graph-embed_amd", "py"))
import ge_amd as ge  # noqa: E402

n = 1_000_000
dev = torch.device("cuda:0")
ctx = ge.Context(0)
rm = ge.rmat_csr(n, 8 * n, seed=12345)
# hub-free: ring lattice with 16 neighbours per vertex
k = 8
cols = (np.arange(n)[:, None] + np.concatenate([np.arange(-k, 0), np.arange(1, k + 1)])) % n
cols.sort(axis=1)
lat = (np.arange(0, n * 2 * k + 1, 2 * k, dtype=np.int32), cols.reshape(-1).astype(np.int32),
       np.ones(n * 2 * k))
for name, A in (("rmat", rm), ("lattice", lat)):
    ip, ix, dx = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in A)
    X = torch.from_numpy(ge.uniform_stream(1, n * 3).reshape(n, 3)).to(dev)
    Y = torch.zeros_like(X)
    print(name, "max deg", int(np.diff(A[0]).max()), flush=True)
    for med, heavy in ((32, 2048), (32, 512), (32, 1024), (32, 4096), (16, 1024), (64, 2048)):
        os.environ["GE_ROWS_MED"] = str(med)
        os.environ["GE_ROWS_HEAVY"] = str(heavy)
        plan = ctx.fa_plan(n, len(A[1]), ip.data_ptr(), ix.data_ptr(), dx.data_ptr(), 3, 0, n)
        plan.set_profiling(True)
        for _ in range(3):
            plan.step(X.data_ptr(), Y.data_ptr())
        ctx.sync()
        _, att_ms, _ = plan.kernel_ms()
        print(f"  med={med} heavy={heavy}: attraction {att_ms:.3f} ms", flush=True)
        plan.close()
