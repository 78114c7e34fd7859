"""Time the coarsest-level persistent kernel on the committed production-size fixture
(tests/golden/fa_coarsest_1e5.npz: an R-MAT LCC coarsened twice by partition(A, 0.125),
n = 1067 with weights and self-loops, as C4's coarsest level) for ITERS iterations,
once per GE_FA_PACK_ROWS value in ROWS (default "4 6"), same process, and check that
every run gives the same bits."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "graph-embed_amd", "py"))
import ge_amd as ge  # noqa: E402

g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "fa_coarsest_1e5.npz"))
A = (g["A_ip"], g["A_ix"], g["A_dx"])
n = len(A[0]) - 1
its = int(os.environ.get("ITERS", "30000"))
ctx = ge.Context(0)
ctx.force_atlas(A, 3, iterations=200, seed=1)  # warm-up
res = []
for rows in os.environ.get("ROWS", "4 6").split():
    os.environ["GE_FA_PACK_ROWS"] = rows
    for rep in range(2):
        t = time.perf_counter()
        x = ctx.force_atlas(A, 3, iterations=its, seed=int(g["seed"]))
        dt = time.perf_counter() - t
        res.append(x)
        print(f"rows {rows}: n={n} nnz={len(A[1])} max deg={int(np.diff(A[0]).max())} "
              f"{its} iterations {dt:.3f} s ({1e6 * dt / its:.2f} us/iteration)", flush=True)
print("bit-identical:", all(np.array_equal(res[0], r) for r in res))
