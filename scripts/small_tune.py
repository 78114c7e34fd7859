"""Time the one-workgroup strict kernel (coarsest level) per lanes-per-row G."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "graph-embed_amd", "py"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import ge_amd as ge  # noqa: E402
import graphs as G  # noqa: E402

ctx = ge.Context(0)
for n, m in [(127, 2500), (127, 8000), (300, 6000), (600, 12000)]:
    A = G.largest_component(G.rmat(n, m, seed=1))
    nn = len(A[0]) - 1
    X0 = G.random_coords(nn, 3, seed=2)
    ref = None
    for g, u in [(g, u) for g in (1, 2, 4, 8, 16) for u in (1,)]:
        if nn * g > 1024:
            continue
        os.environ["GE_SMALL_G"] = str(g)
        os.environ["GE_SMALL_U"] = str(u)
        ctx.force_atlas(A, 3, coords=X0, iterations=10)
        t = time.perf_counter()
        X = ctx.force_atlas(A, 3, coords=X0, iterations=10000)
        dt = time.perf_counter() - t
        same = ref is None or np.array_equal(X, ref)
        ref = X if ref is None else ref
        print(f"n={nn} nnz={len(A[1])} G={g} U={u}: {1e6 * dt / 10000:.2f} us/iteration same={same}",
              flush=True)
