"""Time the C2 attraction pass (classed_rows_kernel<FaRows>) per row layout
(GE_ROWS_TILES) and degree-class bounds (GE_ROWS_MED / GE_ROWS_HEAVY), on the 1M R-MAT and on a hub-free graph."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "graph-embed_amd", "py"))
import ge_amd as ge  # noqa: E402

n = 1_000_000
dev = torch.device("cuda:0")
ctx = ge.Context(0)
rm = ge.rmat_csr(n, 8 * n, seed=12345)
# hub-free: ring lattice with 16 neighbours per vertex
k = 8
cols = (np.arange(n)[:, None] + np.concatenate([np.arange(-k, 0), np.arange(1, k + 1)])) % n
cols.sort(axis=1)
lat = (np.arange(0, n * 2 * k + 1, 2 * k, dtype=np.int32), cols.reshape(-1).astype(np.int32),
       np.ones(n * 2 * k))
def star(n, k, seed):
    """hub 0 joined to k leaves (random ids if seed, else 1..k); the rest isolated"""
    leaves = (np.sort(np.random.RandomState(seed).choice(np.arange(1, n), k, replace=False))
              if seed else np.arange(1, k + 1))
    deg = np.zeros(n, np.int64)
    deg[0] = k
    deg[leaves] = 1
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    ix = np.zeros(ip[-1], np.int32)
    ix[:k] = leaves
    ix[ip[leaves]] = 0
    return ip, ix, np.ones(ip[-1])


graphs = {"rmat": rm, "lattice": lat, "star": star(n, 38455, 0), "star_rand": star(n, 38455, 7)}
for name in os.environ.get("GE_TUNE_GRAPHS", "rmat,lattice").split(","):
    A = graphs[name]
    ip, ix, dx = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in A)
    X = torch.from_numpy(ge.uniform_stream(1, n * 3).reshape(n, 3)).to(dev)
    Y = torch.zeros_like(X)
    print(name, "max deg", int(np.diff(A[0]).max()), flush=True)
    cfgs = ((1, 32, 1024), (1, 32, 512), (1, 32, 256), (0, 32, 1024), (0, 32, 2048))
    if os.environ.get("GE_TUNE_CONFIGS"):  # "tiles,med,heavy;..."
        cfgs = [tuple(int(v) for v in c.split(",")) for c in os.environ["GE_TUNE_CONFIGS"].split(";")]
    extra = [dict(kv.split("=") for kv in c.split(",") if kv) for c in
             os.environ.get("GE_TUNE_ENVS", "").split(";")]
    cfgs = [(c, e) for c in cfgs for e in extra]
    for (tiles, med, heavy), env in cfgs:
        for k in ("GE_ROWS_SERIAL", "GE_TILE_GRID", "GE_ROWS_SEGMENTS"):
            os.environ.pop(k, None)
        os.environ.update(env)
        os.environ["GE_ROWS_TILES"] = str(tiles)
        os.environ["GE_ROWS_MED"] = str(med)
        os.environ["GE_ROWS_HEAVY"] = str(heavy)
        plan = ctx.fa_plan(n, len(A[1]), ip.data_ptr(), ix.data_ptr(), dx.data_ptr(), 3, 0, n)
        for _ in range(2):  # warm-up (code objects, caches)
            plan.step(X.data_ptr(), Y.data_ptr())
        ctx.sync()
        plan.set_profiling(True)
        for _ in range(5):
            plan.step(X.data_ptr(), Y.data_ptr())
        ctx.sync()
        _, att_ms, _ = plan.kernel_ms()
        print(f"  tiles={tiles} med={med} heavy={heavy} {env}: attraction {att_ms:.3f} ms", flush=True)
        plan.close()
