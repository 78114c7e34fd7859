"""Per-iteration time of forceAtlas (strict) for coarsest-level sizes."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "graph-embed_amd", "py"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import ge_amd as ge  # noqa: E402
import graphs as G  # noqa: E402

ctx = ge.Context(0)
cases = [(16, 60), (40, 200), (127, 4000), (500, 10000), (600, 12000), (1068, 30000), (2000, 60000), (5000, 150000)]
if os.environ.get("COARSE_ONLY"):
    cases = [c for c in cases if str(c[0]) in os.environ["COARSE_ONLY"].split(",")]
for n, m in cases:
    A = G.largest_component(G.rmat(n, m, seed=1))
    nn = len(A[0]) - 1
    X0 = G.random_coords(nn, 3, seed=2)
    ctx.force_atlas(A, 3, coords=X0, iterations=10)
    it = 2000
    t = time.perf_counter()
    ctx.force_atlas(A, 3, coords=X0, iterations=it)
    dt = time.perf_counter() - t
    print(f"n={nn} nnz={len(A[1])} small_max={os.environ.get('GE_SMALL_MAX', '-')}: "
          f"{1e6 * dt / it:.1f} us/iteration", flush=True)
