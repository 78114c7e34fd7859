"""The sweep chain in isolation: one streamed aggregate of s members (T = s / 64 row
tiles) alone on the GPU, every row tile a symmetric sweep (GE_FAML_SYM_CHAIN=0), so
the launch is a single convoy of T sweeps.  Prints per s the repulsion launch time
and the lag per sweep (launch / T) -- the tile-time of a chain with the rest of the
GPU idle (round 6: 43 us per sweep at T = 656, profiles/r06/chain_micro_ring.log; the
register-flow variant measured against it is described in DESIGN.md 5d).

usage: python scripts/sym_chain_micro.py [s ...]     (default 4096 16384 41984)
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import ge_amd as ge  # noqa: E402
import graphs as G  # noqa: E402


def main():
    os.environ["GE_FAML_SYM_CHAIN"] = "0"
    sizes = [int(x) for x in sys.argv[1:]] or [4096, 16384, 41984]
    ctx = ge.Context(0)
    dev = torch.device("cuda:0")
    iters = int(os.environ.get("ITERS", "3"))
    for s in sizes:
        A = G.rmat(s, 8 * s, seed=s)
        pip = np.array([0, s], np.int32)
        pix = np.arange(s, dtype=np.int32)
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        d = dict(ip=T(A[0]), ix=T(A[1]), dx=T(A[2]), pip=T(pip), pix=T(pix),
                 vA=T(np.zeros(s, np.int32)), cA=T(np.zeros(3)), rA=T(np.array([0.5])),
                 init=T(ge.uniform_stream(5, s * 3)))
        X = torch.zeros((s, 3), dtype=torch.float64, device=dev)
        p = ge.FamlPlan(ctx, s, d["ip"].data_ptr(), d["ix"].data_ptr(), d["dx"].data_ptr(), pip,
                        d["pip"].data_ptr(), d["pix"].data_ptr(), d["vA"].data_ptr(), 3,
                        iterations=iters)
        p.run(d["cA"].data_ptr(), d["rA"].data_ptr(), d["init"].data_ptr(), X.data_ptr())
        ctx.sync()
        p.set_profiling(True)
        p.run(d["cA"].data_ptr(), d["rA"].data_ptr(), d["init"].data_ptr(), X.data_ptr())
        ctx.sync()
        ms = p.repulse_ms()[0]
        tiles = (s + 63) // 64
        print(json.dumps({"s": s, "tiles": tiles, "schedule": p.schedule(), "repulse_ms": ms,
                          "us_per_sweep": ms * 1e3 / tiles,
                          "us_per_step_on_chain": ms * 1e3 / (3 * s)}), flush=True)
        p.close()
    ctx.close()


if __name__ == "__main__":
    main()
