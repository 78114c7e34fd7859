"""Generates tests/golden/partition_c3_digest.json: the oracle's partition
hierarchy of configs[2]'s graph (LCC of the R-MAT with 1M ids, 8M draws, seed
12345), as level sizes + sha256 of the P_T arrays.  The oracle
(oracle/ge_oracle.cpp, the reference loop of src/partitioner.cpp:1550-1893 restated
with its std::map adjacency) takes ~21 minutes on 8 cores here, so only the digest
is committed; tests/test_partition_device.py::test_partition_device_c3_digest
checks the device hierarchy against it.

usage: python tests/golden/make_partition_digest.py
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


def main():
    O.build()
    n_ids, draws, seed, cf = 1_000_000, 8_000_000, 12345, 0.125
    L = ge.largest_component(ge.rmat_csr(n_ids, draws, seed=seed))
    t = time.time()
    ho = O.partition(L, cf)
    el = time.time() - t
    h = hashlib.sha256()
    for ip, ix, _, _ in ho:
        h.update(np.ascontiguousarray(ip, dtype=np.int32).tobytes())
        h.update(np.ascontiguousarray(ix, dtype=np.int32).tobytes())
    out = {"n_ids": n_ids, "draws": draws, "seed": seed, "cf": cf, "lcc_n": len(L[0]) - 1,
           "lcc_nnz": len(L[1]), "rows": [x[2] for x in ho], "sha256": h.hexdigest(),
           "oracle_seconds": round(el, 1), "generator": "tests/golden/make_partition_digest.py"}
    with open(os.path.join(HERE, "partition_c3_digest.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
