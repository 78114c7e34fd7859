"""Generate tests/golden/faml_c4_level0_100it.npz: C4's level 0 at the embed's
horizon, pinned to the oracle (VERDICT r05 "next" item 2).

    python tests/golden/make_c4_level0_100.py      # ~35 min on 8 threads here

configs[3] (C4, the headline) runs forceAtlasMultilevel with iterations = 100 on
level 0 (src/embed.cpp:793, include/forceatlas.hpp:314-574).  Until round 5 the
oracle checked C4 level 0 for 2 iterations only; the 100-iteration horizon was
covered by agreement among the device's own schedules.  This script evaluates the
oracle (oracle/ge_oracle.cpp orc_force_atlas_ml_aggs, test infrastructure; its
rows are independent, so the thread count does not change the bits) for the full
100 iterations on a sample of level-0 aggregates:

* the largest aggregate (41 930 members, 656 row tiles: the longest sweep chain);
* the two smallest streamed aggregates and the two largest LDS-resident ones (the
  streamed / resident boundary: res_cap = 4096 members at C4, d = 3);
* three aggregates of 2000-4000 members, four of 200-2000 (the resident size
  classes) and 100 random aggregates of <= 200 members.

Inputs are regenerated from seeds, exactly as tests/test_gpu_configs.py builds
them: the 10M-id / 80M-draw R-MAT (seed 12345) and its LCC, partition(A, 0.125)
by the oracle (orc_partition_flat; its hierarchy digest equals the committed
tests/golden/partition_c4_digest.json, which the device partition is checked
against), coords_A / r_A from uniform streams 7 / 8, draw seed 5.  The fixture
stores only the sampled aggregates (ids, sizes, a sha256 of their member lists)
and the oracle's coordinates of their members.

Parity with the reference binary is unpinned: the oracle is a
restatement checked against tests/pyref.py.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))
sys.path.insert(0, os.path.dirname(HERE))

import ge_amd as ge  # noqa: E402
import oracle_lib as O  # noqa: E402

ITERATIONS = 100
SEED = 5
RES_CAP = 4096  # ge_faml.hip faml_plan_build: min(sqrt(W / CUs / 4), large_cap(3)) at C4


def sample_aggregates(PT):
    """The sampled level-0 aggregates (the GPU test re-derives the same list)."""
    sizes = np.diff(PT[0])
    order = np.argsort(sizes, kind="stable")
    streamed = [int(a) for a in order if sizes[a] > RES_CAP]
    resident = [int(a) for a in order if sizes[a] <= RES_CAP]
    big = [int(order[-1])] + streamed[:2] + resident[-2:]
    mid = [int(a) for a in order if 2000 < sizes[a] <= 4000][:3]
    split = [int(a) for a in order if 200 <= sizes[a] <= 2000][-4:]
    small = np.random.default_rng(4).choice(np.nonzero(sizes <= 200)[0], 100, replace=False)
    return np.array(sorted(set(big) | set(mid) | set(split) | set(small.tolist())), np.int32)


def members_sha(PT, aggs):
    h = hashlib.sha256()
    for a in aggs:
        h.update(np.ascontiguousarray(PT[1][PT[0][a]:PT[0][a + 1]], np.int32).tobytes())
    return h.hexdigest()


def main():
    O.build()
    t0 = time.time()
    L = ge.largest_component(ge.rmat_csr(10_000_000, 80_000_000, seed=12345))
    print(f"[{time.time() - t0:6.0f}s] C4 LCC n={len(L[0]) - 1} nnz={len(L[1])}", flush=True)
    hier = O.partition(L, 0.125, flat=True)
    with open(os.path.join(HERE, "partition_c4_digest.json")) as f:
        dig = json.load(f)
    PT = hier[0]
    lvl0 = hashlib.sha256(np.ascontiguousarray(PT[0], np.int32).tobytes() +
                          np.ascontiguousarray(PT[1], np.int32).tobytes()).hexdigest()
    assert lvl0 == dig["level_sha256"][0], "oracle partition differs from the committed digest"
    print(f"[{time.time() - t0:6.0f}s] oracle partition: level 0 equals the digest", flush=True)
    del hier
    m = PT[2]
    vA = O.vertex_of(PT)
    cA = ge.uniform_stream(7, m * 3).reshape(m, 3)
    rA = 0.01 + 0.19 * (ge.uniform_stream(8, m) + 1.0) / 2.0
    aggs = sample_aggregates(PT)
    sizes = np.diff(PT[0])
    print(f"[{time.time() - t0:6.0f}s] {len(aggs)} aggregates, sizes "
          f"{sorted(sizes[aggs].tolist())[-8:]}", flush=True)
    t = time.time()
    X = O.force_atlas_ml_aggs(L, PT, vA, cA, rA, 3, aggs, iterations=ITERATIONS, seed=SEED,
                              nthreads=os.cpu_count())
    print(f"[{time.time() - t0:6.0f}s] oracle {ITERATIONS} iterations in {time.time() - t:.0f} s",
          flush=True)
    rows = np.concatenate([PT[1][PT[0][a]:PT[0][a + 1]] for a in aggs]).astype(np.int64)
    x = X[rows]
    assert np.isfinite(x).all()
    path = os.path.join(HERE, "faml_c4_level0_100it.npz")
    np.savez_compressed(path, aggs=aggs, sizes=sizes[aggs].astype(np.int32),
                        members_sha256=np.array(members_sha(PT, aggs)),
                        level0_sha256=np.array(lvl0), iterations=np.array(ITERATIONS),
                        seed=np.array(SEED), rows=rows.astype(np.int32), x=x)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
