"""configs[4] (C5) device partition alone, with progress notes (GE_PROGRESS): the
100M-id / 800M-draw R-MAT's LCC built on the device, then partition(A, 0.125)."""
import os
import sys
import time

os.environ.setdefault("GE_PROGRESS", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))
import ge_amd as ge  # noqa: E402


def main():
    ctx = ge.Context(0)
    t0 = time.perf_counter()
    L = ctx.rmat_csr(100_000_000, 800_000_000, seed=12345, lcc=True)
    print(f"LCC n={len(L[0]) - 1} nnz={len(L[1])} {time.perf_counter() - t0:.1f}s", flush=True)
    t0 = time.perf_counter()
    hier = ctx.partition(L, 0.125)
    print(f"partition {time.perf_counter() - t0:.1f}s levels {[h[2] for h in hier]}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
