"""Sweep lanes-per-row (GE_GRP_G) and light-row bound (GE_ROWS_MED) at small n."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "graph-embed_amd", "py"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import ge_amd as ge  # noqa: E402
import graphs as G  # noqa: E402

ctx = ge.Context(0)
for n, m in [(600, 12000), (2000, 60000)]:
    A = G.largest_component(G.rmat(n, m, seed=1))
    nn = len(A[0]) - 1
    X0 = G.random_coords(nn, 3, seed=2)
    for g in ("4", "8", "16", "32", "64"):
        for med in ("32", "4", "0"):
            os.environ["GE_GRP_G"] = g
            os.environ["GE_ROWS_MED"] = med
            ctx.force_atlas(A, 3, coords=X0, iterations=10)
            t = time.perf_counter()
            ctx.force_atlas(A, 3, coords=X0, iterations=1000)
            dt = time.perf_counter() - t
            print(f"n={nn} G={g} med={med}: {1e3 * dt:.1f} us/iteration", flush=True)
