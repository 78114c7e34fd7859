"""Device partition at configs' sizes: time it and compare with the host path.

usage: python scripts/partition_dev_check.py N DRAWS [--host] [--levels L]
Prints one JSON line (time, rows per level, sha256 of the P_T arrays).
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))
import ge_amd as ge  # noqa: E402


def digest(h):
    d = hashlib.sha256()
    for ip, ix, _, _ in h:
        d.update(np.ascontiguousarray(ip, dtype=np.int32).tobytes())
        d.update(np.ascontiguousarray(ix, dtype=np.int32).tobytes())
    return d.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", type=int)
    ap.add_argument("draws", type=int)
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--cf", type=float, default=0.125)
    ap.add_argument("--host", action="store_true", help="also run the host path and compare")
    a = ap.parse_args()
    t0 = time.perf_counter()
    L = ge.largest_component(ge.rmat_csr(a.n, a.draws, seed=a.seed))
    t_gen = time.perf_counter() - t0
    ctx = ge.Context(0)
    t0 = time.perf_counter()
    hd = ctx.partition(L, a.cf)
    t_dev = time.perf_counter() - t0
    out = {"n": len(L[0]) - 1, "nnz": len(L[1]), "gen_s": t_gen, "device_s": t_dev,
           "rows": [h[2] for h in hd], "sha256": digest(hd)}
    print(json.dumps(out), flush=True)
    if a.host:
        t0 = time.perf_counter()
        hh = ge.partition(L, a.cf)
        out["host_s"] = time.perf_counter() - t0
        out["host_sha256"] = digest(hh)
        out["equal"] = out["host_sha256"] == out["sha256"]
        print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
