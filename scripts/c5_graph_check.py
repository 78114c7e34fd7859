"""configs[4] (C5) graph: the device R-MAT + LCC against the host generator
(ge_rmat_csr + ge_largest_component), and the CSR properties the device partition
needs (rows strictly ascending, symmetric, unit weights), reported per check."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))
import ge_amd as ge  # noqa: E402


def main():
    ctx = ge.Context(0)
    t0 = time.perf_counter()
    ip, ix, dx = ctx.rmat_csr(100_000_000, 800_000_000, seed=12345, lcc=True)
    n = len(ip) - 1
    print(f"device LCC n={n} nnz={len(ix)} {time.perf_counter() - t0:.1f}s", flush=True)
    row = np.repeat(np.arange(n, dtype=np.int64), np.diff(ip))
    asc = np.diff(ix.astype(np.int64)) > 0
    starts = ip[1:-1]
    asc[starts[starts < len(asc) + 1] - 1] = True  # the row boundaries
    print("rows strictly ascending:", bool(asc.all()), "unit weights:", bool((dx == 1.0).all()),
          "self loops:", int((row == ix).sum()), flush=True)
    key = row * n + ix
    tkey = ix.astype(np.int64) * n + row
    del row
    tkey.sort()
    print("symmetric:", bool(np.array_equal(key, tkey)), flush=True)
    del key, tkey
    t0 = time.perf_counter()
    H = ge.largest_component(ge.rmat_csr(100_000_000, 800_000_000, seed=12345))
    print(f"host LCC {time.perf_counter() - t0:.1f}s equal:",
          all(np.array_equal(a, b) for a, b in zip(H, (ip, ix, dx))), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
