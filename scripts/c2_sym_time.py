"""C2 (configs[1]) single-level repulsion: the symmetric sweeps (ge_sym.hpp, one
aggregate of ceil(n / 64) row tiles) against the ordered-pair kernel
fa_repulse_strict (GE_FA_SYM=0), same bits.  Prints the per-step repulsion and
attraction times of each (HIP events inside libge) and whether the coordinates
after the timed steps are identical.

usage: python scripts/c2_sym_time.py [steps] [n_ids] [draws]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "graph-embed_amd", "py"))
import ge_amd as ge  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n_ids = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
draws = int(sys.argv[3]) if len(sys.argv) > 3 else 8 * n_ids


def main():
    import torch
    ctx = ge.Context(0)
    A = ctx.rmat_csr(n_ids, draws, seed=12345)
    n, nnz = len(A[0]) - 1, len(A[1])
    dev = torch.device("cuda", 0)
    ip, ix, dx = (torch.from_numpy(a).to(dev) for a in A)
    X0 = torch.from_numpy(ge.uniform_stream(12345, n * 3).reshape(n, 3)).to(dev)
    out = {}
    for sym in ("1", "0"):
        os.environ["GE_FA_SYM"] = sym
        plan = ctx.fa_plan(n, nnz, ip.data_ptr(), ix.data_ptr(), dx.data_ptr(), 3, 0, n)
        buf = [X0.clone(), torch.zeros_like(X0)]
        plan.step(buf[0].data_ptr(), buf[1].data_ptr())  # warm-up
        torch.cuda.synchronize()
        buf = [X0.clone(), torch.zeros_like(X0)]
        plan.set_profiling(True)
        t = time.perf_counter()
        for _ in range(steps):
            plan.step(buf[0].data_ptr(), buf[1].data_ptr())
            buf.reverse()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / steps
        rep, att, k = plan.kernel_ms()
        plan.close()
        out[sym] = buf[0].cpu().numpy()
        name = "symmetric sweeps" if sym == "1" else "fa_repulse_strict"
        print(f"{name}: n={n} nnz={nnz} {1e3 * dt:.1f} ms/step, repulsion {rep:.1f} ms, "
              f"attraction {att:.3f} ms ({k} steps)", flush=True)
    print("bit-identical:", bool(np.array_equal(out["0"], out["1"])))
    ctx.close()


if __name__ == "__main__":
    main()
