"""Generates tests/golden/partition_<cfg>_digest.json: the oracle's partition
hierarchy of a configs[] graph as level sizes + sha256 of the P_T arrays.

  c3  configs[2]: LCC of the R-MAT with 1M ids, 8M draws, seed 12345
      (~21 minutes serial here, 2025; the scan is OpenMP-parallel like the
      reference's :1703 since round 3)
  c4  configs[3]: LCC of the R-MAT with 10M ids, 80M draws, seed 12345
      (--flat: 22 minutes on 5 threads here; the std::map oracle ~18 h)

The oracle (oracle/ge_oracle.cpp, the reference loop of src/partitioner.cpp:1550-1893
restated with its std::map adjacency) is far too slow to run inside a test at
these sizes, so only the digest is committed;
tests/test_partition_device.py::test_partition_device_<cfg>_digest checks the
device hierarchy against it.  The per-level sha256 values let a mismatch be
localised to the first differing level.

usage: python tests/golden/make_partition_digest.py [c3|c4] [--host | --flat]

--host: the library's host path (csrc/ge_partition.cpp: the same rounds with
incremental rescans, bit-exact with the oracle on every fixture) instead of the
oracle.  The oracle restates the reference's rescan of every untouched vertex in
every pass (:1703-1726), which at C4 runs ~5 s per round for 9 969 rounds (measured
here: 1 000 rounds in 2 h on 6 threads), so the C4 digest comes from the host path,
pinned first by reproducing the oracle's committed C3 digest in the same run.

--flat (round 5): the oracle's own loop with the per-vertex std::map replaced by
unordered entry lists (orc_partition_flat: every operation in the same order, only
the container differs; tests/test_oracle.py::test_partition_flat_equals_map).  It first
reproduces the committed C3 digest of the std::map oracle, then runs the C4 graph.
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

import ge_amd as ge  # noqa: E402
import oracle_lib as O  # noqa: E402

CONFIGS = {"c3": (1_000_000, 8_000_000), "c4": (10_000_000, 80_000_000)}


def digest(hier):
    """(whole-hierarchy sha256, per-level sha256 list) of P_T indptr/indices."""
    h = hashlib.sha256()
    per = []
    for lvl in hier:
        ip = np.ascontiguousarray(lvl[0], dtype=np.int32).tobytes()
        ix = np.ascontiguousarray(lvl[1], dtype=np.int32).tobytes()
        h.update(ip)
        h.update(ix)
        per.append(hashlib.sha256(ip + ix).hexdigest())
    return h.hexdigest(), per


def lcc(cfg):
    n_ids, draws = CONFIGS[cfg]
    return ge.largest_component(ge.rmat_csr(n_ids, draws, seed=12345))


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    host = "--host" in sys.argv
    flat = "--flat" in sys.argv
    cfg = args[0] if args else "c3"
    n_ids, draws = CONFIGS[cfg]
    seed, cf = 12345, 0.125
    O.build()
    pinned = None
    if host:
        # the host path must first reproduce the oracle's own C3 digest
        with open(os.path.join(HERE, "partition_c3_digest.json")) as f:
            c3 = json.load(f)
        t = time.time()
        got, _ = digest(ge.partition(lcc("c3"), cf))
        pinned = {"c3_sha256": got, "equals_oracle_c3_digest": got == c3["sha256"],
                  "seconds": round(time.time() - t, 1)}
        print("host path at C3:", pinned, flush=True)
        if got != c3["sha256"]:
            raise SystemExit("host path differs from the oracle at C3")
    if flat and cfg != "c3":
        with open(os.path.join(HERE, "partition_c3_digest.json")) as f:
            c3 = json.load(f)
        t = time.time()
        got, _ = digest(O.partition(lcc("c3"), cf, flat=True))
        pinned = {"c3_sha256": got, "equals_oracle_c3_digest": got == c3["sha256"],
                  "seconds": round(time.time() - t, 1)}
        print("flat oracle at C3:", pinned, flush=True)
        if got != c3["sha256"]:
            raise SystemExit("flat oracle differs from the std::map oracle at C3")
    L = lcc(cfg)
    print(f"{cfg}: LCC n={len(L[0]) - 1} nnz={len(L[1])}", flush=True)
    t = time.time()
    ho = ge.partition(L, cf) if host else O.partition(L, cf, flat=flat)
    el = time.time() - t
    if os.environ.get("GE_DIGEST_SAVE"):  # keep the hierarchy itself (not committed)
        np.savez(os.environ["GE_DIGEST_SAVE"],
                 **{f"{k}{l}": a for l, h in enumerate(ho) for k, a in (("ip", h[0]), ("ix", h[1]))})
    full, per = digest(ho)
    out = {"n_ids": n_ids, "draws": draws, "seed": seed, "cf": cf, "lcc_n": len(L[0]) - 1,
           "lcc_nnz": len(L[1]), "rows": [x[2] for x in ho], "sha256": full,
           "level_sha256": per, "seconds": round(el, 1),
           "threads": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count())),
           "method": ("library host path (csrc/ge_partition.cpp), pinned to the oracle by "
                      "the C3 digest" if host else
                      "oracle (oracle/ge_oracle.cpp orc_partition_flat: the reference loop over "
                      "unordered entry lists)" if flat else
                      "oracle (oracle/ge_oracle.cpp orc_partition)"),
           "generator": f"tests/golden/make_partition_digest.py {cfg}" +
                        (" --host" if host else " --flat" if flat else "")}
    if pinned:
        out["flat_oracle_pin" if flat else "host_path_pin"] = pinned
    with open(os.path.join(HERE, f"partition_{cfg}_digest.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
