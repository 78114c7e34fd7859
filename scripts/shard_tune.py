"""Time one strict repulsion step on rank 0's row shard of an N-GPU split
(rows [0, n/N)), per row-slot count R (GE_REP_R), at C2 size."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "graph-embed_amd", "py"))
import ge_amd as ge  # noqa: E402
from ge_amd.dist import row_shards  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
A = ge.rmat_csr(n, 8 * n, seed=12345)
dev = torch.device("cuda:0")
ip, ix, dx = (torch.from_numpy(a).to(dev) for a in A)
X = torch.from_numpy(ge.uniform_stream(12345, n * 3).reshape(n, 3)).to(dev)
Y = torch.zeros_like(X)
ctx = ge.Context(0)
for world in (1, 2, 4, 8):
    chunk, sh = row_shards(n, world)
    rb, re = sh[0]
    ref = None
    for R in ("auto", "1", "2", "4", "8"):
        if R == "auto":
            os.environ.pop("GE_REP_R", None)
        else:
            os.environ["GE_REP_R"] = R
        plan = ctx.fa_plan(n, len(A[1]), ip.data_ptr(), ix.data_ptr(), dx.data_ptr(), 3, rb, re)
        plan.set_profiling(True)
        plan.step(X.data_ptr(), Y.data_ptr())
        ctx.sync()
        rep_ms, att_ms, _ = plan.kernel_ms()
        out = Y[rb:re].clone()
        same = ref is None or torch.equal(out, ref)
        ref = out if ref is None else ref
        print(f"N={world} rows={re - rb} R={R}: repulsion {rep_ms:.1f} ms "
              f"({(re - rb) * (n - 1) / (rep_ms * 1e-3) / 1e9:.1f} Gpairs/s) same={same}",
              flush=True)
        plan.close()
