"""Device partition of a configs[] graph with the library's own phase timers
(GE_PROFILE_PARTITION: device rounds / host bookkeeping / compactions, list
sizes) and progress notes; CFG=c4 (default) or c5; PROF=0: without the phase
timers (they synchronise after every pass)."""
import os
import sys
import time

if os.environ.get("PROF") == "0":  # plain timing: no per-pass synchronisations
    os.environ.pop("GE_PROFILE_PARTITION", None)
else:
    os.environ.setdefault("GE_PROFILE_PARTITION", "1")
os.environ.setdefault("GE_PROGRESS", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))
import ge_amd as ge  # noqa: E402

SIZES = {"c3": (1_000_000, 8_000_000), "c4": (10_000_000, 80_000_000),
         "c5": (100_000_000, 800_000_000)}


def main():
    n_ids, draws = SIZES[os.environ.get("CFG", "c4")]
    ctx = ge.Context(0)
    L = ctx.rmat_csr(n_ids, draws, seed=12345, lcc=True)
    print(f"LCC n={len(L[0]) - 1} nnz={len(L[1])}", flush=True)
    t0 = time.perf_counter()
    hier = ctx.partition(L, 0.125)
    print(f"partition {time.perf_counter() - t0:.2f}s levels {[h[2] for h in hier]}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
