"""Time a coarsest-level forceAtlas (1e5 iterations, src/embed.cpp:586) on a
C4-coarsest-sized graph: the persistent launch against the per-iteration graph
replay (GE_NO_PERSIST=1), same bits.  MODES=persistent,... picks the modes."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "graph-embed_amd", "py"))
import graphs as G  # noqa: E402
import ge_amd as ge  # noqa: E402

n_target = int(sys.argv[1]) if len(sys.argv) > 1 else 1068
its = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
A = G.largest_component(G.rmat(int(n_target * 1.25), 8 * n_target, seed=4))
n = len(A[0]) - 1
ctx = ge.Context()
X0 = G.random_coords(n, 3, seed=1)
ctx.force_atlas(A, 3, coords=X0, iterations=200)  # warm-up (module load, allocations)
res = {}
for mode in os.environ.get("MODES", "persistent,persistent-nopack,graph").split(","):
    if mode == "persistent-nopack":  # 64 lanes per row: one wave per row, not packed
        os.environ["GE_FA_PACKED"] = "0"
    if mode == "graph":
        os.environ.pop("GE_FA_PACKED", None)
        os.environ["GE_NO_PERSIST"] = "1"
    t = time.perf_counter()
    res[mode] = ctx.force_atlas(A, 3, coords=X0, iterations=its)
    dt = time.perf_counter() - t
    print(f"{mode}: n={n} nnz={len(A[1])} iterations={its} {dt:.3f} s "
          f"({1e6 * dt / its:.2f} us/iteration)", flush=True)
print("bit-identical:", all(np.array_equal(next(iter(res.values())), r) for r in res.values()))
