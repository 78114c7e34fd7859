"""A/B timing of the device partition on one graph, interleaved in one process:
`partition(A, 0.125)` with the environment switch ENV=VALUE (argv[1], e.g.
GE_PART_NO_PRESCAN=1) and without it, ROUNDS times each; also checks that both
give the same hierarchy.  CFG=c3 / c4 (default)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))
import ge_amd as ge  # noqa: E402

SIZES = {"c3": (1_000_000, 8_000_000), "c4": (10_000_000, 80_000_000)}


def main():
    key, val = sys.argv[1].split("=", 1)
    n_ids, draws = SIZES[os.environ.get("CFG", "c4")]
    ctx = ge.Context(0)
    L = ctx.rmat_csr(n_ids, draws, seed=12345, lcc=True)
    print(f"LCC n={len(L[0]) - 1} nnz={len(L[1])}", flush=True)
    ref = None
    for r in range(int(os.environ.get("ROUNDS", "2"))):
        for on in (False, True):
            if on:
                os.environ[key] = val
            else:
                os.environ.pop(key, None)
            t0 = time.perf_counter()
            hier = ctx.partition(L, 0.125)
            dt = time.perf_counter() - t0
            same = ref is None or all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
                                      for a, b in zip(hier, ref))
            ref = ref or hier
            print(f"{key}={'set' if on else 'unset'}: {dt:.3f} s, levels {[h[2] for h in hier]}, "
                  f"same hierarchy: {same}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
