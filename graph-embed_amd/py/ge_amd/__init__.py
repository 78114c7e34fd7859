"""ctypes binding of libge.so (include/ge.h) -- the host-side mirror of
graph-embed's partition:: API for Python callers, tests and the benchmark.

The library is the product: every call below runs the gfx950 HIP kernels (or,
for the host-resident steps, the library's own C++).  There is no CPU fallback:
if libge.so is missing or no device is visible, the device entry points raise.

Reference interfaces mirrored (LLNL/graph-embed):
  force_atlas        partition::forceAtlas          include/forceatlas.hpp:89-312
  force_atlas_ml     partition::forceAtlasMultilevel include/forceatlas.hpp:314-574
  partition          partition::partition (hierarchy) src/partitioner.cpp:1550-1893
  interpolation_matrix                               src/partitioner.cpp:29-65
  ptap               P_T.Mult(A).Mult(P_T.Transpose()) examples/embed.cpp:96-98
  embed              partition::embed                src/embed.cpp:561-796
  modularity         partition::modularity           src/partitioner.cpp:69-114
"""
import ctypes
import os
import subprocess

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REPO_ROOT = os.path.dirname(PKG_ROOT)
# GE_LIB_PATH: a variant build of the same library (kernel tuning scripts only)
LIB_PATH = os.environ.get("GE_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libge.so")
HEADER = os.path.join(REPO_ROOT, "include", "ge.h")

MODE_STRICT = 0
MODE_FAST = 1

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_vp = ctypes.c_void_p
_ip = ctypes.POINTER(ctypes.c_int)


class GeError(RuntimeError):
    pass


class FaParams(ctypes.Structure):
    _fields_ = [(k, ctypes.c_double) for k in
                ("ks", "ksmax", "repel", "attract", "gravity", "delta", "tolerate")] + \
               [(k, ctypes.c_int) for k in ("use_weights", "linlog", "nohubs", "normalize")] + \
               [("seed", ctypes.c_uint), ("mode", ctypes.c_int)]


_SIGS = {
    "ge_fa_params_default": (None, [ctypes.POINTER(FaParams)]),
    "ge_last_error": (ctypes.c_char_p, []),
    "ge_version": (ctypes.c_char_p, []),
    "ge_device_count": (ctypes.c_int, [_ip]),
    "ge_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "ge_ctx_destroy": (ctypes.c_int, [_vp]),
    "ge_ctx_set_stream": (ctypes.c_int, [_vp, _vp]),
    "ge_ctx_sync": (ctypes.c_int, [_vp]),
    "ge_force_atlas": (ctypes.c_int, [_vp, ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int,
                                      _f64p, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(FaParams)]),
    "ge_fa_plan_create": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp, _vp, _vp,
                                         ctypes.c_int, ctypes.POINTER(FaParams), ctypes.c_int,
                                         ctypes.c_int, ctypes.POINTER(_vp)]),
    "ge_fa_plan_step": (ctypes.c_int, [_vp, _vp, _vp]),
    "ge_fa_plan_attract": (ctypes.c_int, [_vp, _vp, _vp, _vp]),
    "ge_fa_plan_set_profiling": (ctypes.c_int, [_vp, ctypes.c_int]),
    "ge_fa_plan_kernel_ms": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_double), _ip]),
    "ge_fa_plan_destroy": (ctypes.c_int, [_vp]),
    "ge_force_atlas_ml": (ctypes.c_int, [_vp, ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int,
                                         _i32p, _i32p, _i32p, _f64p, _f64p, _f64p, ctypes.c_int,
                                         ctypes.c_int, ctypes.POINTER(FaParams)]),
    "ge_partition": (ctypes.c_int, [_vp, ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_double,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                    ctypes.c_int, ctypes.POINTER(_vp)]),
    "ge_hier_levels": (ctypes.c_int, [_vp, _ip]),
    "ge_hier_shape": (ctypes.c_int, [_vp, ctypes.c_int, _ip, _ip]),
    "ge_hier_copy": (ctypes.c_int, [_vp, ctypes.c_int, _i32p, _i32p]),
    "ge_hier_free": (ctypes.c_int, [_vp]),
    "ge_interpolation_matrix": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _i32p, _i32p,
                                               ctypes.POINTER(_vp)]),
    "ge_ptap": (ctypes.c_int, [_vp, ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int, _i32p,
                               _i32p, ctypes.POINTER(_vp)]),
    "ge_csr_shape": (ctypes.c_int, [_vp, _ip, _ip, ctypes.POINTER(ctypes.c_longlong)]),
    "ge_csr_copy": (ctypes.c_int, [_vp, _i32p, _vp, _vp]),
    "ge_csr_free": (ctypes.c_int, [_vp]),
    "ge_modularity_device": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp, ctypes.c_int, _vp,
                                            ctypes.POINTER(ctypes.c_double)]),
    "ge_modularity": (ctypes.c_int, [ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int, _i32p,
                                     ctypes.POINTER(ctypes.c_double)]),
    "ge_embed": (ctypes.c_int, [_vp, ctypes.c_int, _i32p, _i32p, _i32p, _i32p, _i32p, _f64p,
                                _i32p, _i32p, _i32p, _i32p, _i32p, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_int, ctypes.POINTER(FaParams), _f64p]),
    "ge_radius_step": (ctypes.c_int, [ctypes.c_int, _f64p, _f64p, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, _vp, _vp, _vp, _vp, _vp, _vp]),
    "ge_uniform_stream": (ctypes.c_int, [ctypes.c_uint, ctypes.c_longlong, _f64p]),
    "ge_faml_plan_create": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp, ctypes.c_int, _i32p,
                                           _vp, _vp, _vp, ctypes.c_int, ctypes.POINTER(FaParams),
                                           ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(_vp)]),
    "ge_faml_plan_create_subset": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp, ctypes.c_int,
                                                  _i32p, _vp, _vp, _vp, ctypes.c_int,
                                                  ctypes.POINTER(FaParams), ctypes.c_int, _i32p,
                                                  ctypes.c_int, ctypes.POINTER(_vp)]),
    "ge_faml_plan_create_shard": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _vp, _vp, _vp,
                                                 ctypes.c_int, _i32p, _vp, _vp, _vp, ctypes.c_int,
                                                 ctypes.POINTER(FaParams), ctypes.c_int, _i32p,
                                                 ctypes.c_int, _i32p, ctypes.c_int,
                                                 ctypes.POINTER(_vp)]),
    "ge_faml_plan_run": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "ge_faml_plan_set_profiling": (ctypes.c_int, [_vp, ctypes.c_int]),
    "ge_faml_plan_kernel_ms": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double),
                                              ctypes.POINTER(ctypes.c_double), _ip]),
    "ge_faml_plan_repulse_ms": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double), _ip,
                                               ctypes.POINTER(ctypes.c_double)]),
    "ge_faml_plan_schedule": (ctypes.c_int, [_vp, _ip, _ip, _ip, _ip]),
    "ge_faml_plan_rows_ms": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double), _ip,
                                            ctypes.POINTER(ctypes.c_longlong),
                                            ctypes.POINTER(ctypes.c_longlong)]),
    "ge_faml_plan_destroy": (ctypes.c_int, [_vp]),
    "ge_selftest_math": (ctypes.c_int, [_vp, ctypes.c_longlong, ctypes.c_ulonglong,
                                        ctypes.POINTER(ctypes.c_longlong)]),
    "ge_rmat_csr": (ctypes.c_int, [ctypes.c_int, ctypes.c_longlong, ctypes.c_ulonglong,
                                   ctypes.POINTER(_vp)]),
    "ge_largest_component": (ctypes.c_int, [ctypes.c_int, _i32p, _i32p, _f64p,
                                            ctypes.POINTER(_vp)]),
    "ge_radius_step_device": (ctypes.c_int, [_vp, ctypes.c_int, _f64p, _f64p, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, _vp, _vp,
                                             _vp, _ip]),
    "ge_embed_via_minimization": (ctypes.c_int, [ctypes.c_int, _i32p, _i32p, ctypes.c_int, _f64p,
                                                 ctypes.c_int, ctypes.c_uint, ctypes.c_int]),
    "ge_rmat_csr_device": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_longlong, ctypes.c_ulonglong,
                                          ctypes.c_int, ctypes.POINTER(_vp)]),
    "ge_largest_component_device": (ctypes.c_int, [_vp, ctypes.c_int, _i32p, _i32p, _f64p,
                                                   ctypes.POINTER(_vp)]),
    # multi-GPU (ge_dist.hip)
    "ge_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "ge_comm_create": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                      ctypes.POINTER(_vp)]),
    "ge_comm_create_transport": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp,
                                                ctypes.POINTER(_vp)]),
    "ge_comm_info": (ctypes.c_int, [_vp, _ip, _ip, _ip]),
    "ge_comm_destroy": (ctypes.c_int, [_vp]),
    "ge_row_shard": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _ip, _ip, _ip]),
    "ge_allgather_coords": (ctypes.c_int, [_vp, _vp, ctypes.c_longlong, ctypes.c_int]),
    "ge_assign_aggregates": (ctypes.c_int, [ctypes.c_int, _i32p, _i32p, _vp, ctypes.c_int,
                                            _i32p]),
    "ge_assign_aggregates_split": (ctypes.c_int, [ctypes.c_int, _i32p, _i32p, _vp, ctypes.c_int,
                                                  ctypes.c_int, _i32p]),
    "ge_allgather_members": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, _i32p, _i32p,
                                            _i32p]),
    "ge_force_atlas_dist": (ctypes.c_int, [_vp, ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int,
                                           _f64p, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(FaParams)]),
    "ge_force_atlas_ml_dist": (ctypes.c_int, [_vp, ctypes.c_int, _i32p, _i32p, _f64p,
                                              ctypes.c_int, _i32p, _i32p, _i32p, _f64p, _f64p,
                                              _f64p, ctypes.c_int, ctypes.c_int,
                                              ctypes.POINTER(FaParams)]),
    "ge_ptap_dist": (ctypes.c_int, [_vp, ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int, _i32p,
                                    _i32p, ctypes.POINTER(_vp)]),
    "ge_embed_dist": (ctypes.c_int, [_vp, ctypes.c_int, _i32p, _i32p, _i32p, _i32p, _i32p,
                                     _f64p, _i32p, _i32p, _i32p, _i32p, _i32p, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(FaParams), _f64p]),
}

_lib = None


def build():
    """Compile libge.so in-tree (hipcc --offload-arch=gfx950)."""
    subprocess.check_call(["make", "-s", "-C", PKG_ROOT, "-j8"])


def lib():
    global _lib
    if _lib is None:
        # torch ships its own libamdhip64.so.7; two HIP runtimes in one process
        # cannot share the device.  Load torch first (when present) so libge.so
        # binds to the runtime already in the process.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise GeError(f"{LIB_PATH} is missing: build it with `make -C {PKG_ROOT}` "
                          "(no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            # an older variant build (GE_LIB_PATH, tuning A/B only) may lack newer entry
            # points; the product library must export every one (tests/test_host.py)
            if os.environ.get("GE_LIB_PATH") and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        msg = lib().ge_last_error().decode(errors="replace")
        raise GeError(f"libge error {rc}: {msg}")


def params(**kw):
    p = FaParams()
    lib().ge_fa_params_default(ctypes.byref(p))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise TypeError(f"unknown ForceAtlas parameter {k}")
        setattr(p, k, v)
    return p


def device_count():
    c = ctypes.c_int(0)
    _check(lib().ge_device_count(ctypes.byref(c)))
    return c.value


def _csr(A):
    ip, ix, dx = A
    return (np.ascontiguousarray(ip, dtype=np.int32), np.ascontiguousarray(ix, dtype=np.int32),
            np.ascontiguousarray(dx, dtype=np.float64))


class Context:
    """One device + one HIP stream (ge_ctx)."""

    def __init__(self, device=0):
        h = _vp()
        _check(lib().ge_ctx_create(device, ctypes.byref(h)))
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            lib().ge_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr):
        _check(lib().ge_ctx_set_stream(self.h, _vp(stream_ptr) if stream_ptr else None))

    def sync(self):
        _check(lib().ge_ctx_sync(self.h))

    # -- partition (device path) ---------------------------------------------
    def partition(self, A, coarsening_factor, **kw):
        return partition(A, coarsening_factor, ctx=self, **kw)

    # -- ForceAtlas ----------------------------------------------------------
    def force_atlas(self, A, dim, coords=None, iterations=100000, **kw):
        ip, ix, dx = _csr(A)
        n = len(ip) - 1
        X = np.zeros((n, dim)) if coords is None else np.array(coords, dtype=np.float64)
        X = np.ascontiguousarray(X)
        p = params(**kw)
        _check(lib().ge_force_atlas(self.h, n, ip, ix, dx, dim, X.reshape(-1),
                                    int(coords is None), iterations, ctypes.byref(p)))
        return X

    def force_atlas_ml(self, A, PT, vertex_A, coords_A, r_A, dim, iterations=10, **kw):
        ip, ix, dx = _csr(A)
        pip = np.ascontiguousarray(PT[0], dtype=np.int32)
        pix = np.ascontiguousarray(PT[1], dtype=np.int32)
        n = len(ip) - 1
        X = np.zeros((n, dim))
        p = params(**kw)
        _check(lib().ge_force_atlas_ml(
            self.h, n, ip, ix, dx, len(pip) - 1, pip, pix,
            np.ascontiguousarray(vertex_A, dtype=np.int32),
            np.ascontiguousarray(coords_A, dtype=np.float64).reshape(-1),
            np.ascontiguousarray(r_A, dtype=np.float64), X.reshape(-1), dim, iterations,
            ctypes.byref(p)))
        return X

    def modularity(self, A, vertex_A, m):
        """partition::modularity with the O(nnz) pass on the device
        (ge_modularity_device); same bits as the host ge_amd.modularity."""
        import torch
        ip, ix, dx = _csr(A)
        dev = torch.device("cuda", self.device)
        t = [torch.from_numpy(np.ascontiguousarray(a)).to(dev)
             for a in (ip, ix, dx, np.asarray(vertex_A, dtype=np.int32))]
        q = ctypes.c_double()
        _check(lib().ge_modularity_device(self.h, len(ip) - 1, _vp(t[0].data_ptr()),
                                          _vp(t[1].data_ptr()), _vp(t[2].data_ptr()), m,
                                          _vp(t[3].data_ptr()), ctypes.byref(q)))
        return q.value

    def ptap(self, A, PT):
        ip, ix, dx = _csr(A)
        pip = np.ascontiguousarray(PT[0], dtype=np.int32)
        pix = np.ascontiguousarray(PT[1], dtype=np.int32)
        h = _vp()
        _check(lib().ge_ptap(self.h, len(ip) - 1, ip, ix, dx, len(pip) - 1, pip, pix,
                             ctypes.byref(h)))
        return _take_csr(h)

    def embed(self, As, hier, dim, base_iterations=100000, ml_iterations=100,
              print_progress=False, **kw):
        parts = concat_levels(As, hier)
        out = np.empty((len(As[0][0]) - 1, dim))
        p = params(**kw)
        _check(lib().ge_embed(self.h, len(hier), *parts, dim, base_iterations, ml_iterations,
                              int(print_progress), ctypes.byref(p), out.reshape(-1)))
        return out

    def radius_step(self, coords_A, dim, coarse_is_base, PTc=None, coords_Ac=None, r_Ac=None,
                    Ac=None):
        """ge_radius_step_device: returns (r_A, coords_A after the rescale, ran_on_device)."""
        cA = np.array(coords_A, dtype=np.float64, copy=True).reshape(-1)
        m = cA.size // dim
        rA = np.zeros(m)
        keep = []

        def ptr(a, dt):
            if a is None:
                return None
            a = np.ascontiguousarray(a, dtype=dt)
            keep.append(a)
            return a.ctypes.data_as(_vp)

        used = ctypes.c_int(-1)
        mc = 0 if PTc is None else len(PTc[0]) - 1
        _check(lib().ge_radius_step_device(
            self.h, m, cA, rA, dim, int(coarse_is_base), mc,
            ptr(None if PTc is None else PTc[0], np.int32),
            ptr(None if PTc is None else PTc[1], np.int32),
            ptr(coords_Ac, np.float64), ptr(r_Ac, np.float64),
            ptr(None if Ac is None else Ac[0], np.int32),
            ptr(None if Ac is None else Ac[1], np.int32), ctypes.byref(used)))
        return rA, cA.reshape(m, dim), bool(used.value)

    def rmat_csr(self, n, draws, seed=12345, lcc=False):
        """ge_rmat_csr_device: the R-MAT (or its largest component) built on the device."""
        h = _vp()
        _check(lib().ge_rmat_csr_device(self.h, n, draws, seed, int(lcc), ctypes.byref(h)))
        return _take_csr(h)

    def largest_component(self, A):
        ip, ix, dx = _csr(A)
        h = _vp()
        _check(lib().ge_largest_component_device(self.h, len(ip) - 1, ip, ix, dx,
                                                 ctypes.byref(h)))
        return _take_csr(h)

    def selftest_math(self, samples=1 << 24, seed=1):
        bad = ctypes.c_longlong()
        _check(lib().ge_selftest_math(self.h, samples, seed, ctypes.byref(bad)))
        return bad.value

    def fa_plan(self, n, nnz, d_ip, d_ix, d_dx, dim, row_begin, row_end, **kw):
        return FaPlan(self, n, nnz, d_ip, d_ix, d_dx, dim, row_begin, row_end, **kw)


_ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, _vp, _vp, _vp, ctypes.c_ulonglong)


class _Transport(ctypes.Structure):
    _fields_ = [("user", _vp), ("allgather", _ALLGATHER_FN)]


def _torch_allgather(send, recv, nbytes):
    """ge_transport.allgather over the default torch.distributed group (gloo):
    host byte blocks, rank-major."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    if nbytes == 0:
        dist.barrier()
        return
    src = np.ctypeslib.as_array((ctypes.c_ubyte * nbytes).from_address(send))
    dst = np.ctypeslib.as_array((ctypes.c_ubyte * (nbytes * world)).from_address(recv))
    outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(outs, torch.from_numpy(src.copy()))
    for r, t in enumerate(outs):
        dst[r * nbytes:(r + 1) * nbytes] = t.numpy()


class Comm:
    """ge_comm: the library's communicator for one rank (one process per GPU).

    backend "rccl": ncclCommInitRank inside libge; the 128-byte unique id made by
    rank 0 (unique_id()) must be handed to every rank (e.g. broadcast_object_list).
    backend "transport": the library's collectives call back into Python, which
    all-gathers host blocks over torch.distributed's default group (gloo) -- the
    multi-process rehearsal on one GPU and the CPU-side tests."""

    def __init__(self, ctx, nranks, rank, backend="rccl", uid=None):
        self.ctx, self.nranks, self.rank = ctx, nranks, rank
        h = _vp()
        if backend == "rccl":
            assert uid is not None and len(uid) == 128
            _check(lib().ge_comm_create(ctx.h, nranks, rank, bytes(uid), ctypes.byref(h)))
        else:
            def cb(user, send, recv, nbytes):
                try:
                    _torch_allgather(send, recv, int(nbytes))
                    return 0
                except Exception:  # reported to the library as a failed collective
                    import traceback
                    traceback.print_exc()
                    return 1
            self._cb = _ALLGATHER_FN(cb)  # kept alive with the communicator
            self._tp = _Transport(None, self._cb)
            _check(lib().ge_comm_create_transport(ctx.h, nranks, rank,
                                                  ctypes.cast(ctypes.byref(self._tp), _vp),
                                                  ctypes.byref(h)))
        self.h = h

    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(128)
        _check(lib().ge_comm_unique_id(buf))
        return buf.raw

    def info(self):
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(lib().ge_comm_info(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, bool(c.value)

    def close(self):
        if getattr(self, "h", None):
            lib().ge_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def allgather_coords(self, d_x, rows_per_rank, dim):
        _check(lib().ge_allgather_coords(self.h, _vp(d_x), rows_per_rank, dim))

    def allgather_members(self, d_x, dim, PT, owner):
        pip = np.ascontiguousarray(PT[0], dtype=np.int32)
        pix = np.ascontiguousarray(PT[1], dtype=np.int32)
        _check(lib().ge_allgather_members(self.h, _vp(d_x), dim, len(pip) - 1, pip, pix,
                                          np.ascontiguousarray(owner, dtype=np.int32)))

    def force_atlas(self, A, dim, coords=None, iterations=100000, **kw):
        ip, ix, dx = _csr(A)
        n = len(ip) - 1
        X = np.zeros((n, dim)) if coords is None else np.array(coords, dtype=np.float64)
        X = np.ascontiguousarray(X)
        p = params(**kw)
        _check(lib().ge_force_atlas_dist(self.h, n, ip, ix, dx, dim, X.reshape(-1),
                                         int(coords is None), iterations, ctypes.byref(p)))
        return X

    def force_atlas_ml(self, A, PT, vertex_A, coords_A, r_A, dim, iterations=10, **kw):
        ip, ix, dx = _csr(A)
        pip = np.ascontiguousarray(PT[0], dtype=np.int32)
        pix = np.ascontiguousarray(PT[1], dtype=np.int32)
        n = len(ip) - 1
        X = np.zeros((n, dim))
        p = params(**kw)
        _check(lib().ge_force_atlas_ml_dist(
            self.h, n, ip, ix, dx, len(pip) - 1, pip, pix,
            np.ascontiguousarray(vertex_A, dtype=np.int32),
            np.ascontiguousarray(coords_A, dtype=np.float64).reshape(-1),
            np.ascontiguousarray(r_A, dtype=np.float64), X.reshape(-1), dim, iterations,
            ctypes.byref(p)))
        return X

    def ptap(self, A, PT):
        ip, ix, dx = _csr(A)
        pip = np.ascontiguousarray(PT[0], dtype=np.int32)
        pix = np.ascontiguousarray(PT[1], dtype=np.int32)
        h = _vp()
        _check(lib().ge_ptap_dist(self.h, len(ip) - 1, ip, ix, dx, len(pip) - 1, pip, pix,
                                  ctypes.byref(h)))
        return _take_csr(h)

    def embed(self, As, hier, dim, base_iterations=100000, ml_iterations=100,
              print_progress=False, **kw):
        parts = concat_levels(As, hier)
        out = np.empty((len(As[0][0]) - 1, dim))
        p = params(**kw)
        _check(lib().ge_embed_dist(self.h, len(hier), *parts, dim, base_iterations,
                                   ml_iterations, int(print_progress), ctypes.byref(p),
                                   out.reshape(-1)))
        return out


def assign_aggregates_split(PT, indptr, nranks, min_members=-1):
    """ge_assign_aggregates_split: owner per aggregate, -1 for the aggregates split
    by row tiles over all ranks (min_members > 0: every aggregate at least that
    large; 0: none; < 0: the automatic rule)."""
    pip = np.ascontiguousarray(PT[0], dtype=np.int32)
    pix = np.ascontiguousarray(PT[1], dtype=np.int32)
    owner = np.empty(len(pip) - 1, dtype=np.int32)
    ipa = None if indptr is None else np.ascontiguousarray(indptr, dtype=np.int32)
    _check(lib().ge_assign_aggregates_split(len(pip) - 1, pip, pix,
                                            None if ipa is None else ipa.ctypes.data_as(_vp),
                                            nranks, min_members, owner))
    return owner


def assign_aggregates(PT, indptr, nranks):
    """ge_assign_aggregates: the rank of every aggregate (LPT by s(s-1) + the
    members' CSR entries when indptr is given)."""
    pip = np.ascontiguousarray(PT[0], dtype=np.int32)
    pix = np.ascontiguousarray(PT[1], dtype=np.int32)
    owner = np.empty(len(pip) - 1, dtype=np.int32)
    ipa = None if indptr is None else np.ascontiguousarray(indptr, dtype=np.int32)
    _check(lib().ge_assign_aggregates(len(pip) - 1, pip, pix,
                                      None if ipa is None else ipa.ctypes.data_as(_vp), nranks,
                                      owner))
    return owner


def row_shard(n, nranks, rank):
    a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _check(lib().ge_row_shard(n, nranks, rank, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
    return a.value, b.value, c.value


class FamlPlan:
    """Device-resident multilevel level (ge_faml_plan_*): P_T's indptr on the host
    (pt_indptr_host, numpy) plus device pointers for everything else."""

    def __init__(self, ctx, n, d_ip, d_ix, d_dx, pt_indptr_host, d_pt_ip, d_pt_ix, d_vA, dim,
                 iterations=100, agg_range=None, aggs=None, split=None, comm=None, **kw):
        """agg_range=(a0, a1) or aggs=(strictly increasing aggregate ids) restricts
        the plan to those aggregates (one rank's share); default: all.  split (with
        comm): aggregates split by row tiles over comm's ranks
        (ge_faml_plan_create_shard)."""
        self.ctx = ctx
        pip = np.ascontiguousarray(pt_indptr_host, dtype=np.int32)
        m = len(pip) - 1
        p = params(**kw)
        h = _vp()
        if comm is not None:
            ids = np.ascontiguousarray(np.zeros(0) if aggs is None else aggs, dtype=np.int32)
            sp = np.ascontiguousarray(np.zeros(0) if split is None else split, dtype=np.int32)
            _check(lib().ge_faml_plan_create_shard(
                ctx.h, comm.h, n, _vp(d_ip), _vp(d_ix), _vp(d_dx), m, pip, _vp(d_pt_ip),
                _vp(d_pt_ix), _vp(d_vA), dim, ctypes.byref(p), iterations, ids, len(ids), sp,
                len(sp), ctypes.byref(h)))
        elif aggs is not None:
            ids = np.ascontiguousarray(aggs, dtype=np.int32)
            _check(lib().ge_faml_plan_create_subset(
                ctx.h, n, _vp(d_ip), _vp(d_ix), _vp(d_dx), m, pip, _vp(d_pt_ip), _vp(d_pt_ix),
                _vp(d_vA), dim, ctypes.byref(p), iterations, ids, len(ids), ctypes.byref(h)))
        else:
            a0, a1 = agg_range if agg_range else (0, m)
            _check(lib().ge_faml_plan_create(ctx.h, n, _vp(d_ip), _vp(d_ix), _vp(d_dx), m, pip,
                                             _vp(d_pt_ip), _vp(d_pt_ix), _vp(d_vA), dim,
                                             ctypes.byref(p), iterations, a0, a1,
                                             ctypes.byref(h)))
        self.h = h

    def run(self, d_cA, d_rA, d_init, d_x):
        _check(lib().ge_faml_plan_run(self.h, _vp(d_cA), _vp(d_rA), _vp(d_init), _vp(d_x)))

    def set_profiling(self, on):
        _check(lib().ge_faml_plan_set_profiling(self.h, int(on)))

    def kernel_ms(self):
        a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        _check(lib().ge_faml_plan_kernel_ms(self.h, ctypes.byref(a), ctypes.byref(b),
                                            ctypes.byref(c)))
        return a.value, b.value, c.value

    def repulse_ms(self):
        """(average ms of one streamed repulsion launch, launches profiled,
        ordered pairs per launch)"""
        a, c, p = ctypes.c_double(), ctypes.c_int(), ctypes.c_double()
        _check(lib().ge_faml_plan_repulse_ms(self.h, ctypes.byref(a), ctypes.byref(c),
                                             ctypes.byref(p)))
        return a.value, c.value, p.value

    def rows_ms(self):
        """(average ms of one streamed member-row pass, passes profiled, rows, CSR
        entries per pass)"""
        a, c = ctypes.c_double(), ctypes.c_int()
        r, e = ctypes.c_longlong(), ctypes.c_longlong()
        _check(lib().ge_faml_plan_rows_ms(self.h, ctypes.byref(a), ctypes.byref(c),
                                          ctypes.byref(r), ctypes.byref(e)))
        return a.value, c.value, r.value, e.value

    def schedule(self):
        """{sweeps, banded, row_blocks, units}: how the streamed aggregates' repulsion
        is scheduled (ge_faml_plan_schedule)."""
        v = [ctypes.c_int() for _ in range(4)]
        _check(lib().ge_faml_plan_schedule(self.h, *[ctypes.byref(x) for x in v]))
        return dict(zip(("sweeps", "banded", "row_blocks", "units"), (x.value for x in v)))

    def close(self):
        """Destroys the plan; raises GeError when the library reports a failure
        that surfaced only at teardown (e.g. a sweep hand-over wait that timed out
        after the last step).  __del__ swallows it."""
        if self.h:
            h, self.h = self.h, None
            _check(lib().ge_faml_plan_destroy(h))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FaPlan:
    """Device-resident ForceAtlas iteration over rows [row_begin, row_end)
    (ge_fa_plan_*).  Device pointers are raw integers (e.g. tensor.data_ptr())."""

    def __init__(self, ctx, n, nnz, d_ip, d_ix, d_dx, dim, row_begin, row_end, **kw):
        self.ctx = ctx
        p = params(**kw)
        h = _vp()
        _check(lib().ge_fa_plan_create(ctx.h, n, nnz, _vp(d_ip), _vp(d_ix), _vp(d_dx), dim,
                                       ctypes.byref(p), row_begin, row_end, ctypes.byref(h)))
        self.h = h

    def step(self, d_x_cur, d_x_next):
        _check(lib().ge_fa_plan_step(self.h, _vp(d_x_cur), _vp(d_x_next)))

    def attract(self, d_x_cur, d_frep, d_x_next):
        """Attraction + gravity + update alone on supplied repulsion sums
        (ge_fa_plan_attract)."""
        _check(lib().ge_fa_plan_attract(self.h, _vp(d_x_cur), _vp(d_frep), _vp(d_x_next)))

    def set_profiling(self, on):
        _check(lib().ge_fa_plan_set_profiling(self.h, int(on)))

    def kernel_ms(self):
        a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        _check(lib().ge_fa_plan_kernel_ms(self.h, ctypes.byref(a), ctypes.byref(b),
                                          ctypes.byref(c)))
        return a.value, b.value, c.value

    def close(self):
        """Destroys the plan; raises GeError when the library reports a failure
        that surfaced only at teardown (e.g. a sweep hand-over wait that timed out
        after the last step).  __del__ swallows it."""
        if self.h:
            h, self.h = self.h, None
            _check(lib().ge_fa_plan_destroy(h))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _take_csr(h):
    r, c, z = ctypes.c_int(), ctypes.c_int(), ctypes.c_longlong()
    _check(lib().ge_csr_shape(h, ctypes.byref(r), ctypes.byref(c), ctypes.byref(z)))
    ip = np.empty(r.value + 1, dtype=np.int32)
    ix = np.empty(z.value, dtype=np.int32)
    dx = np.empty(z.value, dtype=np.float64)
    _check(lib().ge_csr_copy(h, ip, ix.ctypes.data_as(_vp), dx.ctypes.data_as(_vp)))
    lib().ge_csr_free(h)
    return ip, ix, dx


# -- host-resident entry points (no device needed) ----------------------------

def partition(A, coarsening_factor, printing=False, positive_merging=True, stall=1.0,
              matching_iterations=2, merge_leaves=False, ctx=None):
    """Hierarchy of P_T matrices as (indptr, indices, rows, cols) tuples.  With a
    Context the hierarchy is built on its device (integer weights, symmetric A);
    without one, or for other inputs, by the library's host path."""
    ip, ix, dx = _csr(A)
    h = _vp()
    _check(lib().ge_partition(ctx.h if ctx is not None else None, len(ip) - 1, ip, ix, dx,
                              coarsening_factor, int(printing),
                              int(positive_merging), stall, matching_iterations,
                              int(merge_leaves), ctypes.byref(h)))
    try:
        lv = ctypes.c_int()
        _check(lib().ge_hier_levels(h, ctypes.byref(lv)))
        out = []
        for l in range(lv.value):
            r, c = ctypes.c_int(), ctypes.c_int()
            _check(lib().ge_hier_shape(h, l, ctypes.byref(r), ctypes.byref(c)))
            pip = np.empty(r.value + 1, dtype=np.int32)
            pix = np.empty(c.value, dtype=np.int32)
            _check(lib().ge_hier_copy(h, l, pip, pix))
            out.append((pip, pix, r.value, c.value))
        return out
    finally:
        lib().ge_hier_free(h)


def interpolation_matrix(num_cols, sets):
    offs = np.zeros(len(sets) + 1, dtype=np.int32)
    offs[1:] = np.cumsum([len(s) for s in sets])
    flat = np.ascontiguousarray(np.concatenate([np.asarray(s, dtype=np.int32) for s in sets])
                                if sets else np.zeros(0, np.int32), dtype=np.int32)
    h = _vp()
    _check(lib().ge_interpolation_matrix(num_cols, len(sets), offs, flat, ctypes.byref(h)))
    return _take_csr(h)


def modularity(A, vertex_A, m):
    ip, ix, dx = _csr(A)
    q = ctypes.c_double()
    _check(lib().ge_modularity(len(ip) - 1, ip, ix, dx, m,
                               np.ascontiguousarray(vertex_A, dtype=np.int32), ctypes.byref(q)))
    return q.value


def radius_step(coords_A, dim, coarse_is_base, PTc=None, coords_Ac=None, r_Ac=None, Ac=None):
    """Returns (r_A, coords_A after the rescale)."""
    cA = np.array(coords_A, dtype=np.float64, copy=True).reshape(-1)
    m = cA.size // dim
    rA = np.zeros(m)
    keep = []

    def ptr(a, dt):
        if a is None:
            return None
        a = np.ascontiguousarray(a, dtype=dt)
        keep.append(a)
        return a.ctypes.data_as(_vp)

    mc = 0 if PTc is None else len(PTc[0]) - 1
    _check(lib().ge_radius_step(
        m, cA, rA, dim, int(coarse_is_base), mc,
        ptr(None if PTc is None else PTc[0], np.int32), ptr(None if PTc is None else PTc[1], np.int32),
        ptr(coords_Ac, np.float64), ptr(r_Ac, np.float64),
        ptr(None if Ac is None else Ac[0], np.int32), ptr(None if Ac is None else Ac[1], np.int32)))
    return rA, cA.reshape(m, dim)


def embed_via_minimization(A, dim, coords=None, iterations=10, seed=12345):
    """partition::embedViaMinimization(A, d, coords, ITER) (src/embed.cpp:341-559);
    coords=None draws the reference's random start from mt19937(seed)."""
    ip, ix, _ = _csr(A)
    n = len(ip) - 1
    X = np.zeros((n, dim)) if coords is None else np.array(coords, dtype=np.float64)
    X = np.ascontiguousarray(X)
    _check(lib().ge_embed_via_minimization(n, ip, ix, dim, X.reshape(-1), int(coords is None),
                                           seed, iterations))
    return X


def uniform_stream(seed, count):
    out = np.empty(count, dtype=np.float64)
    _check(lib().ge_uniform_stream(seed, count, out))
    return out


def rmat_csr(n, draws, seed=12345):
    h = _vp()
    _check(lib().ge_rmat_csr(n, draws, seed, ctypes.byref(h)))
    return _take_csr(h)


def largest_component(A):
    ip, ix, dx = _csr(A)
    h = _vp()
    _check(lib().ge_largest_component(len(ip) - 1, ip, ix, dx, ctypes.byref(h)))
    return _take_csr(h)


def vertex_of(PT):
    pip, pix = np.asarray(PT[0]), np.asarray(PT[1])
    v = np.empty(len(pix), dtype=np.int32)
    sizes = np.diff(pip)
    v[pix] = np.repeat(np.arange(len(sizes), dtype=np.int32), sizes)
    return v


def concat_levels(As, hier):
    a_n = np.array([len(a[0]) - 1 for a in As], dtype=np.int32)
    a_off = np.cumsum([0] + [len(a[0]) for a in As])[:-1].astype(np.int32)
    a_nz = np.cumsum([0] + [len(a[1]) for a in As])[:-1].astype(np.int32)
    a_ip = np.concatenate([np.asarray(a[0]) for a in As]).astype(np.int32)
    a_ix = np.concatenate([np.asarray(a[1]) for a in As]).astype(np.int32)
    a_dx = np.concatenate([np.asarray(a[2]) for a in As]).astype(np.float64)
    p_rows = np.array([p[2] for p in hier] + [0], dtype=np.int32)
    p_off = np.cumsum([0] + [len(p[0]) for p in hier]).astype(np.int32)
    p_nz = np.cumsum([0] + [len(p[1]) for p in hier]).astype(np.int32)
    p_ip = np.concatenate([np.asarray(p[0]) for p in hier] + [np.zeros(1)]).astype(np.int32)
    p_ix = np.concatenate([np.asarray(p[1]) for p in hier] + [np.zeros(1)]).astype(np.int32)
    return a_n, a_off, a_nz, a_ip, a_ix, a_dx, p_rows, p_off, p_nz, p_ip, p_ix


def header_symbols():
    """Function names declared in include/ge.h."""
    import re
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(ge_\w+)\s*\(", txt, re.M)))
