"""The C++ drop-in headers (graph-embed_amd/include: partitioner.hpp, embed.hpp,
forceatlas.hpp, ...) compiled into the reference's own driver flow
(examples/embed.cpp:93-102) and checked against the C1 golden fixture."""
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PKG = os.path.join(REPO, "graph-embed_amd")


def build_driver(tmp_path):
    exe = str(tmp_path / "embed_driver")
    cmd = ["g++", "-std=c++14", "-O2", "-Wall", "-Wextra", "-Werror",
           f"-I{PKG}/include", f"-I{PKG}/compat", f"-I{REPO}/include",
           os.path.join(HERE, "cpp", "embed_driver.cpp"), f"-L{PKG}/lib", "-lge",
           f"-Wl,-rpath,{PKG}/lib", "-o", exe]
    subprocess.check_call(cmd)
    return exe


def test_dropin_headers_compile(tmp_path):
    assert os.path.exists(build_driver(tmp_path))


def write_csr(path, A):
    ip, ix, dx = A
    with open(path, "wb") as f:
        np.array([len(ip) - 1, len(ix)], np.int32).tofile(f)
        np.asarray(ip, np.int32).tofile(f)
        np.asarray(ix, np.int32).tofile(f)
        np.asarray(dx, np.float64).tofile(f)


@pytest.mark.gpu
@pytest.mark.parametrize("multilevel_api", [False, True])
def test_dropin_driver_c1(tmp_path, golden, multilevel_api):
    g = golden("embed_c1_er1000_d2")
    exe = build_driver(tmp_path)
    inp, out = str(tmp_path / "a.bin"), str(tmp_path / "x.bin")
    write_csr(inp, (g["A_ip"], g["A_ix"], g["A_dx"]))
    args = [exe, inp, out, "2", str(int(g["seed"]))] + (["ml"] if multilevel_api else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert "embedding layer" in r.stdout  # the reference's progress lines
    X = np.fromfile(out, dtype=np.float64).reshape(-1, 2)
    assert np.array_equal(X, g["coords"])
