"""nls_amd -- Python binding of libnls_amd.so (the MI355X-native C-ABI, include/nls.h).

Mirrors the reference's in-process solver API (device/nlse_solver_dev.hpp,
device/sg_solver_dev.hpp, device/matfunc_{complex,real}.hpp) on top of the
C-ABI with ctypes.  There is no CPU fallback: if the HIP library is missing or
cannot be loaded this module raises at import of the library, and every
compute call goes to the GPU.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

__all__ = [
    "NLSE_CUBIC", "NLSE_CQ", "SG_GAUTSCHI", "NLSE_G2", "KG_GAUTSCHI", "SG_G2", "SG_DOUBLE", "SG_HYPERBOLIC",
    "PHI4", "NLSE_CQ_G2", "REAL_EQUATIONS", "F_EXP_ABS", "F_EXP", "F_COS_SQRT", "F_SINC_SQRT",
    "F_SINC2_SQRT", "F_ID_SQRT", "F_SINC2_HALF", "F_SINC", "MAX_KRYLOV", "NlsError", "Config", "Solver",
    "lib", "lib_path", "rccl_unique_id", "slab_planes", "EXPORTED_SYMBOLS",
]

NLSE_CUBIC, NLSE_CQ, SG_GAUTSCHI, NLSE_G2, KG_GAUTSCHI = 0, 1, 2, 3, 4
# G2 device Gautschi family (nlsolvers/device/include/{sg_single,sg_double,sg_hyperbolic,phi4_single}.cuh)
SG_G2, SG_DOUBLE, SG_HYPERBOLIC, PHI4 = 5, 6, 7, 8
# G2 cubic-quintic (nlsolvers/device/include/nlse_cubic_quintic{.cuh,_dev.hpp}): real sigmas,
# pass sigma1=(s1, 0), sigma2=(s2, 0); m(x) via set_coefficients(m)
NLSE_CQ_G2 = 9
REAL_EQUATIONS = (SG_GAUTSCHI, KG_GAUTSCHI, SG_G2, SG_DOUBLE, SG_HYPERBOLIC, PHI4)
F_EXP_ABS, F_EXP, F_COS_SQRT, F_SINC_SQRT, F_SINC2_SQRT, F_ID_SQRT, F_SINC2_HALF, F_SINC = range(8)
MAX_KRYLOV = 32

EXPORTED_SYMBOLS = (
    "nls_abi_version", "nls_config_default", "nls_create", "nls_destroy", "nls_last_error",
    "nls_local_planes", "nls_comm_size", "nls_set_field", "nls_set_sg_state", "nls_step", "nls_sync",
    "nls_get_field", "nls_get_sg_velocity", "nls_krylov_apply", "nls_laplacian_apply",
    "nls_rccl_unique_id", "nls_group_create", "nls_group_destroy", "nls_set_timing",
    "nls_get_timing", "nls_reset_timing", "nls_set_coefficients", "nls_apply_bc",
    "nls_get_field_async", "nls_wait_field", "nls_host_alloc", "nls_host_free", "nls_slab_planes",
    "nls_step_sewi", "nls_debug_oplog", "nls_debug_knob", "nls_placement",
    "nls_peer_state", "nls_build_info",
)
# nls_debug_oplog entry kinds (include/nls.h enum nls_op_kind)
OP_ALLREDUCE, OP_SEND, OP_RECV, OP_WAIT_HALO, OP_WAIT_COMPUTE, OP_ALLGATHER, OP_DROPPED = 1, 2, 3, 4, 5, 6, 7

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)


def lib_path() -> str:
    return os.environ.get("NLS_AMD_LIB", os.path.join(_PKG, "lib", "libnls_amd.so"))


class Config(C.Structure):
    _fields_ = [
        ("dim", C.c_int32), ("equation", C.c_int32),
        ("nx", C.c_uint32), ("ny", C.c_uint32), ("nz", C.c_uint32),
        ("dx", C.c_double), ("dy", C.c_double),
        ("krylov_m", C.c_uint32),
        ("sigma1", C.c_double * 2), ("sigma2", C.c_double * 2),
        ("device", C.c_int32), ("nranks", C.c_int32), ("rank", C.c_int32),
        ("rccl_id", C.c_void_p), ("local_group", C.c_void_p),
    ]


class Timing(C.Structure):
    _fields_ = [
        ("class_ms", C.c_double * 6), ("class_count", C.c_uint64 * 6),
        ("update_ms", C.c_double * MAX_KRYLOV), ("update_count", C.c_uint64 * MAX_KRYLOV),
        ("steps", C.c_uint64), ("graph_steps", C.c_uint64),
    ]


class NlsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"nls error {code}: {msg}")
        self.code = code


_LIB = None


def lib():
    """Load libnls_amd.so (raises if it is absent -- no fallback path exists)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built: run `make` (or __graft_entry__.build())")
    L = C.CDLL(path)
    H = C.c_void_p
    dp = C.POINTER(C.c_double)
    L.nls_abi_version.restype = C.c_int
    L.nls_config_default.argtypes = [C.POINTER(Config)]
    L.nls_config_default.restype = None
    L.nls_create.argtypes = [C.POINTER(Config), C.POINTER(H)]
    L.nls_destroy.argtypes = [H]
    L.nls_last_error.argtypes = [H]
    L.nls_last_error.restype = C.c_char_p
    L.nls_local_planes.argtypes = [H, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                   C.POINTER(C.c_uint64)]
    L.nls_comm_size.argtypes = [H, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    L.nls_slab_planes.argtypes = [C.c_uint32, C.c_int32, C.c_int32, C.POINTER(C.c_uint32),
                                  C.POINTER(C.c_uint32)]
    L.nls_set_field.argtypes = [H, dp, C.c_uint64]
    L.nls_set_sg_state.argtypes = [H, dp, dp, dp, C.c_uint64]
    L.nls_step.argtypes = [H, C.c_double, C.c_uint32]
    L.nls_step_sewi.argtypes = [H, C.c_double, C.c_uint32]
    L.nls_set_coefficients.argtypes = [H, dp, dp, C.c_uint64]
    L.nls_apply_bc.argtypes = [H]
    L.nls_sync.argtypes = [H]
    L.nls_get_field.argtypes = [H, dp, C.c_uint64]
    L.nls_get_sg_velocity.argtypes = [H, C.c_double, dp, C.c_uint64]
    L.nls_get_field_async.argtypes = [H, dp, C.c_uint64]
    L.nls_wait_field.argtypes = [H]
    L.nls_host_alloc.argtypes = [C.c_uint64, C.POINTER(C.c_void_p)]
    L.nls_host_free.argtypes = [C.c_void_p]
    L.nls_krylov_apply.argtypes = [H, dp, C.c_double, C.c_double, C.c_int32, dp, C.c_uint64]
    L.nls_laplacian_apply.argtypes = [H, dp, dp, C.c_uint64]
    L.nls_rccl_unique_id.argtypes = [C.c_void_p]
    L.nls_group_create.argtypes = [C.c_int32, C.POINTER(C.c_void_p)]
    L.nls_group_destroy.argtypes = [C.c_void_p]
    L.nls_set_timing.argtypes = [H, C.c_int32]
    L.nls_get_timing.argtypes = [H, C.POINTER(Timing)]
    L.nls_reset_timing.argtypes = [H]
    L.nls_debug_oplog.argtypes = [H, C.POINTER(C.c_int32), C.c_uint64, C.POINTER(C.c_uint64)]
    L.nls_debug_knob.argtypes = [H, C.c_int32, C.c_int32]
    L.nls_peer_state.argtypes = [H, C.POINTER(C.c_int32)]
    L.nls_build_info.restype = C.c_char_p
    L.nls_build_info.argtypes = []
    L.nls_placement.argtypes = [H, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_float),
                                C.c_uint32]
    if L.nls_abi_version() != 6:
        raise RuntimeError("libnls_amd ABI mismatch")
    _LIB = L
    return L


def build_info() -> dict:
    """The library's build provenance (nls_build_info): src_sha256, arch, compiler, built."""
    txt = lib().nls_build_info().decode()
    out, key = {}, None
    for tok in txt.split(" "):
        if "=" in tok:
            key, val = tok.split("=", 1)
            out[key] = val
        elif key:
            out[key] += " " + tok
    return out


def sources_sha256() -> str | None:
    """sha256 of the library sources beside this package, in the Makefile's order (sorted
    csrc/*.hip, *.hpp, *.cpp, then include/nls.h); None where they are not present."""
    import glob
    import hashlib
    root = os.path.dirname(_PKG)
    names = sorted(os.path.relpath(p, root) for e in ("hip", "hpp", "cpp")
                   for p in glob.glob(os.path.join(_PKG, "csrc", f"*.{e}")))
    names.append(os.path.join("include", "nls.h"))
    h = hashlib.sha256()
    for n in names:
        try:
            with open(os.path.join(root, n), "rb") as f:
                h.update(f.read())
        except OSError:
            return None
    return h.hexdigest()


def slab_planes(npl: int, nranks: int, rank: int) -> tuple[int, int]:
    """(z0, nzl) of `rank`'s slab -- the library's own decomposition (no device needed)."""
    z0, nzl = C.c_uint32(), C.c_uint32()
    rc = lib().nls_slab_planes(npl, nranks, rank, C.byref(z0), C.byref(nzl))
    if rc != 0:
        raise NlsError(rc, "bad slab arguments")
    return z0.value, nzl.value


def rccl_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    rc = lib().nls_rccl_unique_id(buf)
    if rc != 0:
        raise NlsError(rc, lib().nls_last_error(None).decode())
    return buf.raw


class Group:
    """In-process rank group (nls_group_create): ranks are Solver handles of this
    process driven from separate host threads; halo by D2D copies, fixed-order
    device all-reduce.  Same slab layout and kernels as the RCCL path."""

    def __init__(self, nranks: int):
        g = C.c_void_p()
        rc = lib().nls_group_create(int(nranks), C.byref(g))
        if rc != 0:
            raise NlsError(rc, "nls_group_create failed")
        self._g = g
        self.nranks = nranks

    def close(self):
        if getattr(self, "_g", None):
            lib().nls_group_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Solver:
    """One device handle (nls_handle).

    equation: NLSE_CUBIC / NLSE_CQ / NLSE_G2 (complex128 fields) or SG_GAUTSCHI, KG_GAUTSCHI,
    SG_G2, SG_DOUBLE, SG_HYPERBOLIC, PHI4 (float64).
    NLSE_G2 (nlsolvers/device/include/nlse_dev.hpp) also needs set_coefficients(m, c).
    Grid: dim 2 -> (ny, nx), dim 3 -> (nz, ny, nx); dx, dy as the reference
    drivers compute them (dx = 2 Lx / (nx - 1)).
    """

    def __init__(self, dim, nx, ny, nz=1, dx=1.0, dy=None, equation=NLSE_CUBIC, m=10,
                 sigma1=(0.0, 0.5), sigma2=(-0.5, 0.0), device=-1, nranks=1, rank=0,
                 rccl_id: bytes | None = None, group: "Group | None" = None):
        L = lib()
        cfg = Config()
        L.nls_config_default(C.byref(cfg))
        cfg.dim, cfg.equation = dim, equation
        cfg.nx, cfg.ny, cfg.nz = nx, ny, nz if dim == 3 else 1
        cfg.dx = dx
        cfg.dy = dx if dy is None else dy
        cfg.krylov_m = m
        cfg.sigma1[0], cfg.sigma1[1] = sigma1
        cfg.sigma2[0], cfg.sigma2[1] = sigma2
        cfg.device, cfg.nranks, cfg.rank = device, nranks, rank
        self._id = C.create_string_buffer(rccl_id, 128) if rccl_id else None
        cfg.rccl_id = C.cast(self._id, C.c_void_p) if self._id is not None else None
        self._group = group
        cfg.local_group = group._g if group is not None else None
        self.cfg = cfg
        self.complex = equation not in REAL_EQUATIONS
        self.dtype = np.complex128 if self.complex else np.float64
        h = C.c_void_p()
        rc = L.nls_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise NlsError(rc, L.nls_last_error(None).decode())
        self._h = h
        z0, nzl, nloc = C.c_uint32(), C.c_uint32(), C.c_uint64()
        self._call(L.nls_local_planes, C.byref(z0), C.byref(nzl), C.byref(nloc))
        self.z0, self.nzl, self.n_local = z0.value, nzl.value, nloc.value

    def comm_size(self) -> tuple[int, str]:
        """(ranks, transport) as the handle's transport reports them (nls_comm_size):
        the RCCL communicator's count, the in-process group's size, or (1, "none")."""
        n, tr = C.c_int32(), C.c_int32()
        self._call(lib().nls_comm_size, C.byref(n), C.byref(tr))
        return n.value, ("none", "rccl", "group")[tr.value]

    # -- plumbing ---------------------------------------------------------
    def _call(self, fn, *args):
        rc = fn(self._h, *args)
        if rc != 0:
            raise NlsError(rc, lib().nls_last_error(self._h).decode())
        return rc

    def close(self):
        if getattr(self, "_h", None):
            lib().nls_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _in(self, a, dtype=None):
        a = np.ascontiguousarray(np.asarray(a, dtype=dtype or self.dtype)).ravel()
        if a.size != self.n_local:
            raise NlsError(-2, f"expected {self.n_local} cells, got {a.size}")
        return a.view(np.float64) if np.iscomplexobj(a) else a

    def _out(self, dtype=None):
        return np.empty(self.n_local, dtype=dtype or self.dtype)

    # -- reference API mirror ----------------------------------------------
    def set_field(self, u):
        a = self._in(u)
        self._call(lib().nls_set_field, _dptr(a), self.n_local)

    def set_sg_state(self, u, u_past, mfield=None):
        a, b = self._in(u, np.float64), self._in(u_past, np.float64)
        c = self._in(mfield, np.float64) if mfield is not None else None
        self._call(lib().nls_set_sg_state, _dptr(a), _dptr(b), _dptr(c) if c is not None else None,
                   self.n_local)

    def set_coefficients(self, mfield, cfield=None):
        """G2: focusing field m(x) and anisotropy c(x) of div(c grad u) (local slab);
        NLSE_CQ_G2: m(x) only (cfield None)."""
        a = self._in(mfield, np.float64)
        if cfield is None:
            self._call(lib().nls_set_coefficients, _dptr(a), None, self.n_local)
        else:
            b = self._in(cfield, np.float64)
            self._call(lib().nls_set_coefficients, _dptr(a), _dptr(b), self.n_local)

    def apply_bc(self):
        """Neumann copy BC of the G2 drivers (boundaries.cuh:10-81)."""
        self._call(lib().nls_apply_bc)

    def step_sewi(self, dt, step_number):
        """G2 sEWI step (nlse_dev.hpp:205-238); step_number 1 is an SS2 step."""
        self._call(lib().nls_step_sewi, float(dt), int(step_number))

    def step(self, dt, nsteps=1):
        self._call(lib().nls_step, float(dt), int(nsteps))

    def sync(self):
        self._call(lib().nls_sync)

    def get_field(self):
        out = self._out()
        self._call(lib().nls_get_field, _dptr(out.view(np.float64)), self.n_local)
        return out

    def get_field_async(self, out: np.ndarray):
        """Enqueue a snapshot of the field into `out` (keep it alive and unread
        until wait_field())."""
        if out.dtype != self.dtype or out.size != self.n_local or not out.flags.c_contiguous:
            raise NlsError(-2, "out must be a C-contiguous array of the field dtype and size")
        self._async_out = out
        self._call(lib().nls_get_field_async, _dptr(out.view(np.float64)), self.n_local)

    def wait_field(self):
        self._call(lib().nls_wait_field)
        self._async_out = None

    def get_sg_velocity(self, dt):
        out = self._out(np.float64)
        self._call(lib().nls_get_sg_velocity, float(dt), _dptr(out), self.n_local)
        return out

    def krylov_apply(self, x, t, func):
        a = self._in(x)
        out = self._out()
        t = complex(t)
        self._call(lib().nls_krylov_apply, _dptr(a), t.real, t.imag, int(func),
                   _dptr(out.view(np.float64)), self.n_local)
        return out

    def laplacian(self, x):
        a = self._in(x)
        out = self._out()
        self._call(lib().nls_laplacian_apply, _dptr(a), _dptr(out.view(np.float64)), self.n_local)
        return out

    def set_timing(self, on=True):
        self._call(lib().nls_set_timing, 1 if on else 0)

    def reset_timing(self):
        self._call(lib().nls_reset_timing)

    def oplog(self) -> list[tuple[int, int, int, int]]:
        """Transport operations since the last call, in issue order, as
        (kind, stream, count, peer) (nls_debug_oplog; recorded with NLS_OPLOG=1 at
        creation)."""
        n = C.c_uint64()
        self._call(lib().nls_debug_oplog, None, 0, C.byref(n))  # size only
        buf = (C.c_int32 * (4 * max(1, n.value)))()
        self._call(lib().nls_debug_oplog, buf, n.value, C.byref(n))  # copies and clears
        return [tuple(buf[4 * i:4 * i + 4]) for i in range(n.value)]

    def debug_knob(self, knob: int, value: int):
        """Launch-shape knob of this live handle (nls_debug_knob: 1 tail dynamic tile
        queue, 2 tail tile depth, 3 k_p2d tile order), for same-allocation A/B runs."""
        self._call(lib().nls_debug_knob, int(knob), int(value))

    def peer_state(self) -> str:
        """The boundary-plane transport (nls_peer_state): off / active / fell_back / pending."""
        v = C.c_int32()
        self._call(lib().nls_peer_state, C.byref(v))
        return ("off", "active", "fell_back", "pending")[v.value]

    def placement(self) -> dict:
        """The basis placement chosen at creation (nls_placement): candidates probed,
        the one kept, and each candidate's probe time in ms (n = 0: no probe)."""
        n, k = C.c_int32(), C.c_int32()
        ms = (C.c_float * 8)()
        self._call(lib().nls_placement, C.byref(n), C.byref(k), ms, 8)
        return {"candidates": n.value, "chosen": k.value, "probe_ms": [round(ms[i], 3) for i in range(n.value)]}

    def timing(self) -> dict:
        t = Timing()
        self._call(lib().nls_get_timing, C.byref(t))
        names = ["alpha", "update", "reduce", "pointwise", "halo", "final"]
        return {
            "class_ms": {n: t.class_ms[i] for i, n in enumerate(names)},
            "class_count": {n: int(t.class_count[i]) for i, n in enumerate(names)},
            "update_ms": [t.update_ms[j] for j in range(MAX_KRYLOV)],
            "update_count": [int(t.update_count[j]) for j in range(MAX_KRYLOV)],
            "steps": int(t.steps),
            "graph_steps": int(t.graph_steps),
        }
