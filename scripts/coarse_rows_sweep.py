"""Packed rows per block (GE_FA_PACK_ROWS = 4 / 6) of the coarsest-level persistent
kernel across level sizes: R-MAT LCCs of about N vertices (argv: the sizes), ITERS
iterations each, both settings in one process; prints us per iteration and whether
the two runs gave the same bits."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "graph-embed_amd", "py"))
import graphs as G  # noqa: E402
import ge_amd as ge  # noqa: E402

its = int(os.environ.get("ITERS", "20000"))
ctx = ge.Context()
for nt in [int(x) for x in (sys.argv[1:] or ["1068", "1300", "1600"])]:
    A = G.largest_component(G.rmat(int(nt * 1.25), 8 * nt, seed=4))
    n = len(A[0]) - 1
    X0 = G.random_coords(n, 3, seed=1)
    ctx.force_atlas(A, 3, coords=X0, iterations=200)  # warm-up
    res = {}
    for R in ("4", "6"):
        os.environ["GE_FA_PACK_ROWS"] = R
        t = time.perf_counter()
        res[R] = ctx.force_atlas(A, 3, coords=X0, iterations=its)
        dt = time.perf_counter() - t
        print(f"n={n} rows {R}: {its} iterations {dt:.3f} s ({1e6 * dt / its:.2f} us/iteration)",
              flush=True)
    os.environ.pop("GE_FA_PACK_ROWS")
    print(f"n={n} bit-identical: {np.array_equal(res['4'], res['6'])}", flush=True)
