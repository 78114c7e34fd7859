"""Device R-MAT (+ LCC) against the host generator at large sizes (configs[4] is
100M ids / 800M draws): per size, unit weights, strictly ascending rows, and the
first index where the device arrays differ from the host's."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))
import ge_amd as ge  # noqa: E402


def props(name, A):
    ip, ix, dx = A
    asc = np.diff(ix.astype(np.int64)) > 0
    b = ip[1:-1].astype(np.int64) - 1
    asc[b[(b >= 0) & (b < len(asc))]] = True
    print(f"  {name}: n={len(ip) - 1} nnz={len(ix)} ip[-1]={ip[-1]} unit={bool((dx == 1.0).all())} "
          f"ascending={bool(asc.all())} first_bad_entry={int(np.argmin(asc)) if not asc.all() else -1}",
          flush=True)


def diff(name, a, b):
    if len(a) != len(b):
        print(f"  {name}: lengths {len(a)} vs {len(b)}", flush=True)
        return
    d = np.flatnonzero(a != b)
    print(f"  {name}: {len(d)} differ" + (f", first at {d[0]} ({a[d[0]]} vs {b[d[0]]})"
                                          if len(d) else ""), flush=True)


def main():
    ctx = ge.Context(0)
    for n_ids, draws in [(int(x.split(":")[0]), int(x.split(":")[1]))
                         for x in os.environ.get("SIZES", "100000000:800000000").split(",")]:
        print(f"R-MAT {n_ids} ids {draws} draws", flush=True)
        t0 = time.perf_counter()
        D = ctx.rmat_csr(n_ids, draws, seed=12345)
        print(f"  device {time.perf_counter() - t0:.1f}s", flush=True)
        props("device", D)
        H = ge.rmat_csr(n_ids, draws, seed=12345)
        props("host", H)
        for nm, a, b in zip(("indptr", "indices", "data"), D, H):
            diff(nm, a, b)
        del D
        DL = ctx.rmat_csr(n_ids, draws, seed=12345, lcc=True)
        props("device LCC", DL)
        HL = ge.largest_component(H)
        del H
        for nm, a, b in zip(("LCC indptr", "LCC indices", "LCC data"), DL, HL):
            diff(nm, a, b)
        del DL, HL
    ctx.close()


if __name__ == "__main__":
    main()
