"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py

The reference cannot be built here (linalgcpp is absent and a stand-in is not
allowed) and ships no fixtures, so these vectors are produced by the oracle
(oracle/ge_oracle.cpp), which tests/test_oracle.py cross-checks bit for bit
against the independent pure-Python restatement tests/pyref.py.  Parity of the
fixtures with the reference itself is therefore UNPINNED (Oracle).

Every fixture stores its inputs (graph, seeds, parameters) with the outputs, so
the GPU tests need nothing but the .npz file.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import graphs as G  # noqa: E402
import oracle_lib as O  # noqa: E402


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, sum(a.nbytes for a in arrays.values() if hasattr(a, "nbytes")), "B raw")


def csr_arrays(prefix, A):
    return {prefix + "_ip": np.asarray(A[0], np.int32), prefix + "_ix": np.asarray(A[1], np.int32),
            prefix + "_dx": np.asarray(A[2], np.float64)}


def main():
    # 1. forceAtlas, supplied init, 1 / 10 / 100 iterations
    A = G.erdos_renyi(300, 0.03, seed=11)
    X0 = G.random_coords(300, 3, seed=5)
    outs = {f"x_it{it}": O.force_atlas(A, 3, coords=X0, iterations=it) for it in (1, 10, 100)}
    save("fa_er300_d3", **csr_arrays("A", A), x0=X0, **outs)

    # 2. forceAtlas with random init (mt19937 seed) in 2-D
    B = G.largest_component(G.rmat(700, 4000, seed=8))
    save("fa_rmat_d2_seeded", **csr_arrays("A", B), seed=np.array(2024),
         x_it20=O.force_atlas(B, 2, iterations=20, seed=2024))

    # 3. partition hierarchy + P^T A P of an R-MAT LCC (cf = 0.125)
    C = G.largest_component(G.rmat(4096, 40000, seed=12345))
    hier = O.partition(C, 0.125)
    arrs = csr_arrays("A", C)
    As = O.hierarchy_As(C, hier)
    for l, PT in enumerate(hier):
        arrs[f"P{l}_ip"], arrs[f"P{l}_ix"] = PT[0], PT[1]
        arrs[f"P{l}_shape"] = np.array([PT[2], PT[3]], np.int32)
        arrs.update(csr_arrays(f"A{l + 1}", As[l + 1]))
    arrs["levels"] = np.array(len(hier))
    save("partition_rmat4096", **arrs)

    # 4. one forceAtlasMultilevel level with supplied coords_A / r_A
    PT = hier[0]
    vA = O.vertex_of(PT)
    cA = G.random_coords(PT[2], 3, seed=21)
    rA = np.random.RandomState(22).uniform(0.05, 0.5, PT[2])
    save("faml_rmat4096_l0", **csr_arrays("A", C), P_ip=PT[0], P_ix=PT[1], vA=vA, cA=cA, rA=rA,
         seed=np.array(77), x_it100=O.force_atlas_ml(C, PT, vA, cA, rA, 3, iterations=100,
                                                    seed=77))

    # 5. config 1 end to end: ER(1000, 0.01), partition(A, 0.1), P^T A P, embed d = 2
    E = G.erdos_renyi(1000, 0.01, seed=42)
    hE = O.partition(E, 0.1)
    AsE = O.hierarchy_As(E, hE)
    arrs = csr_arrays("A", E)
    for l, PT in enumerate(hE):
        arrs[f"P{l}_ip"], arrs[f"P{l}_ix"] = PT[0], PT[1]
        arrs[f"P{l}_shape"] = np.array([PT[2], PT[3]], np.int32)
    arrs["levels"] = np.array(len(hE))
    arrs["seed"] = np.array(12345)
    arrs["coords"] = O.embed(AsE, hE, 2, seed=12345, base_iterations=100000, ml_iterations=100)
    save("embed_c1_er1000_d2", **arrs)


if __name__ == "__main__":
    main()
