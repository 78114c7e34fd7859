"""The linalgcpp graph readers of the compat layer (compat/parser.hpp), which
the reference's drivers call before partition/embed (examples/embed.cpp:80-91).
linalgcpp is not vendored, so the formats are restated and parity is unpinned;
these tests pin each reader against scipy on the same matrix."""
import os
import subprocess

import numpy as np
import pytest
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "graph-embed_amd")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("readers") / "readers")
    subprocess.check_call(["g++", "-std=c++14", "-O1", "-Wall", "-Wextra", "-Werror",
                           f"-I{PKG}/compat", os.path.join(HERE, "cpp", "readers.cpp"), "-o", out])
    return out


def run(exe, *args):
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    head, ip, ix, dx = r.stdout.split("\n")[:4]
    rows, cols, nnz = map(int, head.split())
    return (rows, cols, np.array(ip.split(), int), np.array(ix.split(), int),
            np.array(dx.split(), float))


def as_csr(res):
    rows, cols, ip, ix, dx = res
    return sp.csr_matrix((dx, ix, ip), shape=(rows, cols))


def same(res, M):
    A = as_csr(res)
    M = sp.csr_matrix(M)
    M.sum_duplicates()
    M.sort_indices()
    assert A.shape == M.shape
    assert np.array_equal(A.indptr, M.indptr) and np.array_equal(A.indices, M.indices)
    assert np.array_equal(A.data, M.data)


EDGES = [(0, 1), (1, 2), (2, 0), (3, 1), (1, 2)]  # a duplicate; vertex 3 one-way


@pytest.mark.parametrize("sym", [0, 1])
def test_adjacency_list(exe, tmp_path, sym):
    p = tmp_path / "g.adj"
    p.write_text("".join(f"{i} {j}\n" for i, j in EDGES) + "\n")
    I, J = map(np.array, zip(*EDGES))
    M = sp.coo_matrix((np.ones(len(I)), (I, J)), shape=(4, 3)).tocsr()
    if sym:
        M = sp.coo_matrix((np.ones(len(I)), (I, J)), shape=(4, 4))
        M = (M + M.T).tocsr()
    same(run(exe, "adjlist", p, sym), M)


@pytest.mark.parametrize("sym", [0, 1])
def test_coordinate_list_and_writer(exe, tmp_path, sym):
    p = tmp_path / "g.coo"
    vals = [0.5, 2.0, -1.25, 3.0, 0.1]
    p.write_text("".join(f"{i} {j} {v!r}\n" for (i, j), v in zip(EDGES, vals)))
    I, J = map(np.array, zip(*EDGES))
    n = 4 if sym else None
    M = sp.coo_matrix((vals, (I, J)), shape=(4, 4) if sym else (4, 3))
    if sym:
        M = M + M.T
    same(run(exe, "coolist", p, sym), M.tocsr())
    out = tmp_path / "back.coo"
    first = run(exe, "writecoo", p, sym, out)
    assert n is None or first[0] == n
    same(run(exe, "coolist", out, 0), as_csr(first))


def test_table(exe, tmp_path):
    p = tmp_path / "g.table"
    p.write_text("1 2\n\n0 3 3\n2\n")
    M = sp.csr_matrix((np.ones(6), ([0, 0, 2, 2, 2, 3], [1, 2, 0, 3, 3, 2])), shape=(4, 4))
    same(run(exe, "table", p), M)


def test_csr(exe, tmp_path):
    rs = np.random.RandomState(3)
    M = sp.random(7, 5, density=0.4, random_state=rs, format="csr")
    p = tmp_path / "g.csr"
    p.write_text(f"7 5 {M.nnz}\n" + " ".join(map(str, M.indptr)) + "\n" +
                 " ".join(map(str, M.indices)) + "\n" + " ".join(repr(float(v)) for v in M.data) + "\n")
    same(run(exe, "csr", p), M)


@pytest.mark.parametrize("kind", ["real general", "pattern symmetric", "integer symmetric"])
def test_matrix_market(exe, tmp_path, kind):
    p = tmp_path / "g.mtx"
    ents = [(1, 1, 4.0), (2, 1, 1.5), (3, 2, -2.0), (4, 3, 7.0)]
    if kind.startswith("integer"):
        ents = [(i, j, float(int(v))) for i, j, v in ents]
    body = "".join(f"{i} {j}\n" if kind.startswith("pattern") else f"{i} {j} {v!r}\n"
                   for i, j, v in ents)
    p.write_text(f"%%MatrixMarket matrix coordinate {kind}\n% comment\n4 4 {len(ents)}\n" + body)
    I = np.array([e[0] - 1 for e in ents])
    J = np.array([e[1] - 1 for e in ents])
    V = np.ones(len(ents)) if kind.startswith("pattern") else np.array([e[2] for e in ents])
    M = sp.coo_matrix((V, (I, J)), shape=(4, 4))
    if "symmetric" in kind:
        off = I != J
        M = M + sp.coo_matrix((V[off], (J[off], I[off])), shape=(4, 4))
    same(run(exe, "mtx", p), M.tocsr())


def test_reader_errors(exe, tmp_path):
    bad = tmp_path / "bad.mtx"
    bad.write_text("%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n")
    r = subprocess.run([exe, "mtx", str(bad)], capture_output=True, text=True)
    assert r.returncode == 1 and "coordinate" in r.stderr
    r = subprocess.run([exe, "adjlist", str(tmp_path / "missing")], capture_output=True, text=True)
    assert r.returncode == 1 and "cannot open" in r.stderr
