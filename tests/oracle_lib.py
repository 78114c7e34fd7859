"""ctypes binding of oracle/liboracle.so (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


class FaParams(ctypes.Structure):
    _fields_ = [(k, ctypes.c_double) for k in
                ("ks", "ksmax", "repel", "attract", "gravity", "delta", "tolerate")] + \
               [(k, ctypes.c_int) for k in ("use_weights", "linlog", "nohubs", "normalize")]


def build():
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = ctypes.CDLL(ORACLE_SO)
        L.orc_fa_params_default.argtypes = [ctypes.POINTER(FaParams)]
        L.orc_uniform_stream.argtypes = [ctypes.c_uint, ctypes.c_longlong, _f64p]
        L.orc_degrees.argtypes = [ctypes.c_int, _i32p, _f64p, ctypes.c_int, _f64p]
        L.orc_force_atlas.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int, _f64p,
                                      ctypes.c_int, ctypes.c_uint, ctypes.c_int,
                                      ctypes.POINTER(FaParams), ctypes.c_int]
        L.orc_fa_forces_rows.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int, _f64p,
                                         _f64p, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(FaParams), _f64p, ctypes.c_int]
        L.orc_fa_step_rows.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int, _f64p,
                                       _f64p, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(FaParams), _f64p, _f64p, ctypes.c_int]
        L.orc_force_atlas_ml.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int, _i32p,
                                         _i32p, _i32p, _f64p, _f64p, _f64p, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_uint, ctypes.POINTER(FaParams),
                                         ctypes.c_int]
        L.orc_fa_step_rows_frep.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int,
                                            _f64p, _f64p, ctypes.c_int, ctypes.c_int,
                                            ctypes.POINTER(FaParams), _f64p, _f64p, _f64p,
                                            ctypes.c_int]
        L.orc_force_atlas_ml_aggs.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int,
                                              _i32p, _i32p, _i32p, _f64p, _f64p, _f64p,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_uint,
                                              ctypes.POINTER(FaParams), _i32p, ctypes.c_int,
                                              ctypes.c_int]
        L.orc_partition.restype = ctypes.c_void_p
        L.orc_partition.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_double,
                                    ctypes.c_int, ctypes.c_double, ctypes.c_int]
        L.orc_partition_flat.restype = ctypes.c_void_p
        L.orc_partition_flat.argtypes = L.orc_partition.argtypes
        L.orc_hier_levels.argtypes = [ctypes.c_void_p]
        L.orc_hier_shape.argtypes = [ctypes.c_void_p, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.orc_hier_copy.argtypes = [ctypes.c_void_p, ctypes.c_int, _i32p, _i32p]
        L.orc_hier_free.argtypes = [ctypes.c_void_p]
        L.orc_modularity.restype = ctypes.c_double
        L.orc_modularity.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int, _i32p]
        L.orc_ptap.restype = ctypes.c_void_p
        L.orc_ptap.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int, _i32p, _i32p]
        L.orc_csr_shape.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                    ctypes.POINTER(ctypes.c_int)]
        L.orc_csr_copy.argtypes = [ctypes.c_void_p, _i32p, _i32p, _f64p]
        L.orc_csr_free.argtypes = [ctypes.c_void_p]
        L.orc_embed.argtypes = [ctypes.c_int, _i32p, _i32p, _i32p, _i32p, _i32p, _f64p,
                                _i32p, _i32p, _i32p, _i32p, _i32p, ctypes.c_int, ctypes.c_uint,
                                ctypes.c_int, ctypes.c_int, _f64p, ctypes.c_int]
        L.orc_embed_via_minimization.argtypes = [ctypes.c_int, _i32p, _i32p, ctypes.c_int, _f64p,
                                                 ctypes.c_int, ctypes.c_uint, ctypes.c_int]
        L.orc_embed_via_minimization_ml.argtypes = [
            ctypes.c_int, _i32p, _i32p, _i32p, _i32p, _i32p, _f64p, _i32p, _i32p, _i32p, _i32p,
            _i32p, ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f64p,
            ctypes.c_int]
        L.orc_radius_step.argtypes = [ctypes.c_int, _f64p, _f64p, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, _i32p, _i32p]
        _lib = L
    return _lib


def params(**kw):
    p = FaParams()
    lib().orc_fa_params_default(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _csr(A):
    ip, ix, dx = A
    return (np.ascontiguousarray(ip, dtype=np.int32), np.ascontiguousarray(ix, dtype=np.int32),
            np.ascontiguousarray(dx, dtype=np.float64))


def uniform_stream(seed, count):
    out = np.empty(count, dtype=np.float64)
    lib().orc_uniform_stream(seed, count, out)
    return out


def degrees(A, use_weights=True):
    ip, ix, dx = _csr(A)
    n = len(ip) - 1
    out = np.empty(n, dtype=np.float64)
    lib().orc_degrees(n, ip, dx, int(use_weights), out)
    return out


def force_atlas(A, dim, coords=None, iterations=100000, seed=0, nthreads=0, **kw):
    ip, ix, dx = _csr(A)
    n = len(ip) - 1
    X = np.zeros((n, dim)) if coords is None else np.array(coords, dtype=np.float64, copy=True)
    X = np.ascontiguousarray(X)
    p = params(**kw)
    rc = lib().orc_force_atlas(n, ip, ix, dx, dim, X.reshape(-1), int(coords is None), seed,
                               iterations, ctypes.byref(p), nthreads)
    assert rc == 0
    return X


def fa_forces_rows(A, coords, deg, rb, re, nthreads=0, **kw):
    ip, ix, dx = _csr(A)
    n = len(ip) - 1
    dim = coords.shape[1]
    out = np.empty((re - rb, dim))
    p = params(**kw)
    rc = lib().orc_fa_forces_rows(n, ip, ix, dx, dim, np.ascontiguousarray(coords).reshape(-1),
                                  np.ascontiguousarray(deg), rb, re, ctypes.byref(p),
                                  out.reshape(-1), nthreads)
    assert rc == 0
    return out


def fa_step_rows(A, coords, deg, rb, re, fprev_rows, coords_next, nthreads=0, **kw):
    """One iteration for a row shard; fprev_rows and coords_next are updated in place."""
    ip, ix, dx = _csr(A)
    p = params(**kw)
    rc = lib().orc_fa_step_rows(len(ip) - 1, ip, ix, dx, coords.shape[1],
                                np.ascontiguousarray(coords).reshape(-1), deg, rb, re,
                                ctypes.byref(p), fprev_rows.reshape(-1), coords_next.reshape(-1),
                                nthreads)
    assert rc == 0


def fa_step_rows_frep(A, coords, deg, rb, re, frep_rows, fprev_rows, coords_next, nthreads=0,
                      **kw):
    """fa_step_rows with the rows' repulsion sums supplied (frep_rows)."""
    ip, ix, dx = _csr(A)
    p = params(**kw)
    rc = lib().orc_fa_step_rows_frep(len(ip) - 1, ip, ix, dx, coords.shape[1],
                                     np.ascontiguousarray(coords).reshape(-1), deg, rb, re,
                                     ctypes.byref(p), np.ascontiguousarray(frep_rows).reshape(-1),
                                     fprev_rows.reshape(-1), coords_next.reshape(-1), nthreads)
    assert rc == 0


def force_atlas_ml_aggs(A, PT, vertex_A, coords_A, r_A, dim, aggs, iterations=100, seed=0,
                        nthreads=0, **kw):
    """force_atlas_ml evaluated for the aggregates `aggs` only (same draw stream); the
    rows of other aggregates stay 0."""
    ip, ix, dx = _csr(A)
    pip = np.ascontiguousarray(PT[0], dtype=np.int32)
    pix = np.ascontiguousarray(PT[1], dtype=np.int32)
    n = len(ip) - 1
    X = np.zeros((n, dim))
    p = params(**kw)
    ag = np.ascontiguousarray(aggs, dtype=np.int32)
    rc = lib().orc_force_atlas_ml_aggs(n, ip, ix, dx, len(pip) - 1, pip, pix,
                                       np.ascontiguousarray(vertex_A, dtype=np.int32),
                                       np.ascontiguousarray(coords_A, dtype=np.float64).reshape(-1),
                                       np.ascontiguousarray(r_A, dtype=np.float64), X.reshape(-1),
                                       dim, iterations, seed, ctypes.byref(p), ag, len(ag),
                                       nthreads)
    assert rc == 0
    return X


def force_atlas_ml(A, PT, vertex_A, coords_A, r_A, dim, iterations=100, seed=0, nthreads=0,
                   **kw):
    ip, ix, dx = _csr(A)
    pip = np.ascontiguousarray(PT[0], dtype=np.int32)
    pix = np.ascontiguousarray(PT[1], dtype=np.int32)
    n = len(ip) - 1
    m = len(pip) - 1
    X = np.zeros((n, dim))
    p = params(**kw)
    rc = lib().orc_force_atlas_ml(n, ip, ix, dx, m, pip, pix,
                                  np.ascontiguousarray(vertex_A, dtype=np.int32),
                                  np.ascontiguousarray(coords_A, dtype=np.float64).reshape(-1),
                                  np.ascontiguousarray(r_A, dtype=np.float64), X.reshape(-1), dim,
                                  iterations, seed, ctypes.byref(p), nthreads)
    assert rc == 0
    return X


def partition(A, cf, positive_merging=True, stall=1.0, matching=2, flat=False):
    """Returns a list of P_T as (indptr, indices, rows, cols).  flat: the same loop
    over unordered entry lists (orc_partition_flat: identical results, for C4)."""
    ip, ix, dx = _csr(A)
    L = lib()
    fn = L.orc_partition_flat if flat else L.orc_partition
    h = fn(len(ip) - 1, ip, ix, dx, cf, int(positive_merging), stall, matching)
    out = []
    for l in range(L.orc_hier_levels(h)):
        r, c = ctypes.c_int(), ctypes.c_int()
        L.orc_hier_shape(h, l, ctypes.byref(r), ctypes.byref(c))
        pip = np.empty(r.value + 1, dtype=np.int32)
        pix = np.empty(c.value, dtype=np.int32)
        L.orc_hier_copy(h, l, pip, pix)
        out.append((pip, pix, r.value, c.value))
    L.orc_hier_free(h)
    return out


def modularity(A, vertex_A, m):
    ip, ix, dx = _csr(A)
    return lib().orc_modularity(len(ip) - 1, ip, ix, dx, m,
                                np.ascontiguousarray(vertex_A, dtype=np.int32))


def ptap(A, PT):
    ip, ix, dx = _csr(A)
    pip = np.ascontiguousarray(PT[0], dtype=np.int32)
    pix = np.ascontiguousarray(PT[1], dtype=np.int32)
    L = lib()
    h = L.orc_ptap(len(ip) - 1, ip, ix, dx, len(pip) - 1, pip, pix)
    r, z = ctypes.c_int(), ctypes.c_int()
    L.orc_csr_shape(h, ctypes.byref(r), ctypes.byref(z))
    oip = np.empty(r.value + 1, dtype=np.int32)
    oix = np.empty(z.value, dtype=np.int32)
    odx = np.empty(z.value, dtype=np.float64)
    L.orc_csr_copy(h, oip, oix, odx)
    L.orc_csr_free(h)
    return oip, oix, odx


def vertex_of(PT):
    pip, pix = PT[0], PT[1]
    v = np.empty(len(pix), dtype=np.int32)
    for a in range(len(pip) - 1):
        v[pix[pip[a]:pip[a + 1]]] = a
    return v


def hierarchy_As(A, hier):
    As = [_csr(A)]
    for PT in hier:
        As.append(ptap(As[-1], PT))
    return As


def _concat_levels(As, hier):
    a_n = np.array([len(a[0]) - 1 for a in As], dtype=np.int32)
    a_off = np.cumsum([0] + [len(a[0]) for a in As])[:-1].astype(np.int32)
    a_nz = np.cumsum([0] + [len(a[1]) for a in As])[:-1].astype(np.int32)
    a_ip = np.concatenate([a[0] for a in As]).astype(np.int32)
    a_ix = np.concatenate([a[1] for a in As]).astype(np.int32)
    a_dx = np.concatenate([a[2] for a in As]).astype(np.float64)
    p_rows = np.array([p[2] for p in hier] + [0], dtype=np.int32)
    p_off = np.cumsum([0] + [len(p[0]) for p in hier])[:-1].astype(np.int32) \
        if hier else np.zeros(1, np.int32)
    p_nz = np.cumsum([0] + [len(p[1]) for p in hier])[:-1].astype(np.int32) \
        if hier else np.zeros(1, np.int32)
    p_ip = np.concatenate([p[0] for p in hier] + [np.zeros(1)]).astype(np.int32)
    p_ix = np.concatenate([p[1] for p in hier] + [np.zeros(1)]).astype(np.int32)
    return a_n, a_off, a_nz, a_ip, a_ix, a_dx, p_rows, p_off, p_nz, p_ip, p_ix


def embed_via_minimization(A, dim, coords=None, iterations=10, seed=0):
    ip, ix, _ = _csr(A)
    n = len(ip) - 1
    X = np.zeros((n, dim)) if coords is None else np.array(coords, dtype=np.float64)
    X = np.ascontiguousarray(X)
    rc = lib().orc_embed_via_minimization(n, ip, ix, dim, X.reshape(-1), int(coords is None),
                                          seed, iterations)
    assert rc == 0, rc
    return X


def embed_via_minimization_ml(As, hier, dim, seed=0, base_iterations=100000, ml_iterations=100,
                              min_iterations=1000, nthreads=0):
    parts = _concat_levels(As, hier)
    out = np.empty((len(As[0][0]) - 1, dim))
    rc = lib().orc_embed_via_minimization_ml(len(hier), *parts, dim, seed, base_iterations,
                                             ml_iterations, min_iterations, out.reshape(-1),
                                             nthreads)
    assert rc == 0, rc
    return out


def embed(As, hier, dim, seed=0, base_iterations=100000, ml_iterations=100, nthreads=0):
    parts = _concat_levels(As, hier)
    n0 = len(As[0][0]) - 1
    out = np.empty((n0, dim))
    rc = lib().orc_embed(len(hier), *parts, dim, seed, base_iterations, ml_iterations,
                         out.reshape(-1), nthreads)
    assert rc == 0, rc
    return out
