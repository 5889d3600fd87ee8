"""ctypes wrappers for the CPU checker -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module.  It wraps
  * oracle/liboracle.so      -- the C restatement of the reference (mg_oracle.c)
  * oracle/_ref/libmgref.so  -- the unmodified reference sources, compiled here
                                (optional: only present where /root/reference
                                was available at build time); libmgref_o3.so
                                is the same sources at -O3 (CPU baseline only)
All arrays are float64 numpy arrays in the reference's row-major (n+1)^2 layout.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libmgref.so")
REF_NU2_PATH = os.path.join(HERE, "_ref", "libmgref_nu2.so")   # NITER = 2 (config 2)
REF_O3_PATH = os.path.join(HERE, "_ref", "libmgref_o3.so")     # -O3 -march=x86-64-v3

_dp = C.POINTER(C.c_double)


def _p(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_dp)


def _load(path):
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built (run `make -C oracle`)")
    return C.CDLL(path)


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load(LIB_PATH)
        L = _lib
        L.or_compute_norm.restype = C.c_double
        L.or_mg_inner.restype = C.c_long
        L.or_mg_outer.restype = C.c_int
        L.or_timestepper.restype = C.c_int
    return _lib


def ref_available(nsmooth: int = 3) -> bool:
    return os.path.exists(REF_NU2_PATH if nsmooth == 2 else REF_PATH)


_refs = {}


def ref(nsmooth: int = 3):
    """The reference library (nsmooth 3 = unmodified; 2 = the NITER=2 build)."""
    global _ref
    if nsmooth not in _refs:
        r = _load(REF_NU2_PATH if nsmooth == 2 else REF_PATH)
        r.ref_compute_norm.restype = C.c_double
        r.ref_vcycle_once.restype = C.c_double
        r.ref_vcycle_once_tower.restype = C.c_double
        r.ref_time_vcycles.restype = C.c_double
        _refs[nsmooth] = r
    if nsmooth == 3:
        _ref = _refs[3]
    return _refs[nsmooth]


D = C.c_double
LNG = C.c_long


# ---------------------------------------------------------------- oracle ops
def set_threads(n: int):
    lib().or_set_threads(C.c_int(n))


def set_fp_mode(fm: int):
    """1: the checker's gauss_seidel / residual in libmgx's fp_mode fma form
    (mg_oracle.h or_set_fp_mode); 0: the reference's term order."""
    lib().or_set_fp_mode(C.c_int(1 if fm else 0))


def compute_rhs(u, n, v1, v2, k, nu, h, rhs=None):
    rhs = np.zeros_like(u) if rhs is None else rhs
    lib().or_compute_rhs(_p(rhs), _p(u), LNG(n), _p(v1), _p(v2), D(k), D(nu), D(h))
    return rhs


def residual(u, rhs, n, v1, v2, k, nu, h, res=None):
    res = np.zeros_like(u) if res is None else res
    lib().or_residual(_p(res), _p(u), _p(rhs), LNG(n), _p(v1), _p(v2), D(k), D(nu), D(h))
    return res


def compute_norm(res, n):
    return lib().or_compute_norm(_p(res), LNG(n))


def gauss_seidel(u, rhs, n, v1, v2, k, nu, h):
    """In place, like gs.cpp:109."""
    lib().or_gauss_seidel(_p(u), _p(rhs), LNG(n), _p(v1), _p(v2), D(k), D(nu), D(h))
    return u


def prolongation(u, n):
    up = np.zeros((2 * n + 1) ** 2, dtype=np.float64)
    lib().or_prolongation(_p(up), _p(u), LNG(n))
    return up


def restriction(up, n):
    u = np.zeros((n // 2 + 1) ** 2, dtype=np.float64)
    lib().or_restriction(_p(u), _p(up), LNG(n))
    return u


def gauss_seidel_slab(u, rhs, n, r0, v1, v2, k, nu, h):
    """gauss_seidel on rows [r0, r0 + rows) held in u (in place); exact on rows
    [r0 + 2, r0 + rows - 3]."""
    nr = u.size // (n + 1)
    lib().or_gauss_seidel_slab(_p(u), _p(rhs), LNG(n), LNG(r0), LNG(nr), _p(v1), _p(v2),
                               D(k), D(nu), D(h))
    return u


def residual_slab(u, rhs, n, r0, v1, v2, k, nu, h):
    """residual on a row slab (zeros where not computed); exact on rows
    [r0 + 1, r0 + rows - 2]."""
    res = np.zeros_like(u)
    nr = u.size // (n + 1)
    lib().or_residual_slab(_p(res), _p(u), _p(rhs), LNG(n), LNG(r0), LNG(nr), _p(v1),
                           _p(v2), D(k), D(nu), D(h))
    return res


def compute_rhs_slab(u, n, r0, v1, v2, k, nu, h):
    rhs = np.zeros_like(u)
    nr = u.size // (n + 1)
    lib().or_compute_rhs_slab(_p(rhs), _p(u), LNG(n), LNG(r0), LNG(nr), _p(v1), _p(v2),
                              D(k), D(nu), D(h))
    return rhs


def prolongation_slab(u, n, c0):
    """Fine rows [2 c0, 2 (c0 + rows - 1)] (clipped to 2n) of prolongation(u)
    from the coarse rows [c0, c0 + rows) held in u."""
    cn = u.size // (n + 1)
    I1 = min(2 * (c0 + cn - 1), 2 * n)
    up = np.zeros((I1 - 2 * c0 + 1) * (2 * n + 1), dtype=np.float64)
    lib().or_prolongation_slab(_p(up), _p(u), LNG(n), LNG(c0), LNG(cn))
    return up


def init_problem(N):
    cnt = (N + 1) ** 2
    u0, v1, v2 = (np.empty(cnt) for _ in range(3))
    lib().or_init_problem(_p(u0), _p(v1), _p(v2), LNG(N))
    return u0, v1, v2


def timestepper(u0, v1, v2, nu, maxlvl, n, dt, T, dx, tol=1e-6, shape=1, nsmooth=3,
                tower_mode=0):
    """multigrid.cpp:124.  Returns (uT, cycles_per_step)."""
    uT = np.empty_like(u0)
    steps = int(T / dt)
    cyc = (C.c_int * max(steps, 1))()
    lib().or_timestepper(_p(uT), _p(u0), _p(v1), _p(v2), D(nu), C.c_int(maxlvl), LNG(n),
                         D(dt), D(T), D(dx), D(tol), C.c_int(shape), C.c_int(nsmooth),
                         C.c_int(tower_mode), cyc)
    return uT, list(cyc)[:steps]


class Tower:
    """Level towers built the way timestepper builds them (multigrid.cpp:131-162)."""

    def __init__(self, u0, v1, v2, n, maxlvl, tower_mode=0):
        self.n, self.maxlvl = n, maxlvl
        P = _dp * (maxlvl + 1)
        self.u, self.v1, self.v2, self.rhs = P(), P(), P(), P()
        self._keep = [u0.copy(), v1.copy(), v2.copy(), np.zeros_like(u0)]
        self.u[0], self.v1[0], self.v2[0], self.rhs[0] = (_p(a) for a in self._keep)
        self.tmp = np.zeros_like(u0)
        lib().or_build_tower(self.v1, self.v2, self.u, self.rhs, C.c_int(maxlvl), LNG(n),
                             C.c_int(tower_mode))

    def level(self, which, lvl):
        n = self.n >> lvl
        ptr = getattr(self, which)[lvl]
        return np.ctypeslib.as_array(ptr, shape=((n + 1) ** 2,)).copy()

    @property
    def ufine(self):
        return self._keep[0]

    @property
    def rhsfine(self):
        return self._keep[3]

    def mg_inner(self, dt, nu, shape=1, nsmooth=3):
        dx = 1.0 / self.n
        return lib().or_mg_inner(self.u, self.rhs, self.v1, self.v2, _p(self.tmp), D(dx),
                                 LNG(self.n), C.c_int(0), C.c_int(self.maxlvl),
                                 C.c_int(shape), D(dt), D(nu), C.c_int(nsmooth))

    def mg_outer(self, dt, nu, tol=1e-6, shape=1, nsmooth=3):
        dx = 1.0 / self.n
        r0, r = D(), D()
        cyc = lib().or_mg_outer(self.u, self.v1, self.v2, self.rhs, _p(self.tmp), D(nu),
                                C.c_int(self.maxlvl), LNG(self.n), D(dt), D(dx), D(tol),
                                C.c_int(shape), C.c_int(nsmooth), C.byref(r0), C.byref(r))
        return cyc, r0.value, r.value

    def close(self):
        if self.maxlvl > 1:
            lib().or_free_tower(self.v1, self.v2, self.u, self.rhs, C.c_int(self.maxlvl))
            self.maxlvl = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ----------------------------------------------------------- reference (_ref)
def ref_timestepper(u0, v1, v2, nu, maxlvl, n, dt, T, dx, tol=1e-6, shape=1, nthreads=1,
                    nsmooth=3):
    uT = np.empty_like(u0)
    a = [x.copy() for x in (u0, v1, v2)]
    ref(nsmooth).ref_timestepper(_p(uT), _p(a[0]), _p(a[1]), _p(a[2]), D(nu), C.c_int(maxlvl),
                          C.c_int(n), D(dt), D(T), D(dx), D(tol), C.c_int(shape),
                          C.c_int(nthreads))
    return uT


def ref_op(name, *args):
    return getattr(ref(), name)(*args)


_ref_o3 = None


def ref_o3_available() -> bool:
    return os.path.exists(REF_O3_PATH)


def ref_o3():
    """The unmodified reference sources built -O3 (timing only, never a checker)."""
    global _ref_o3
    if _ref_o3 is None:
        _ref_o3 = _load(REF_O3_PATH)
        _ref_o3.ref_time_vcycles.restype = C.c_double
    return _ref_o3


def ref_time_vcycles(n, maxlvl, nu, cycles, nthreads, opt="O0"):
    """Seconds for `cycles` reference V-cycles (+ residual/norm) at size n on
    `nthreads` OpenMP threads; opt "O0" = the reference Makefile flags, "O3"."""
    setup, res = D(), D()
    t = (ref_o3() if opt == "O3" else ref()).ref_time_vcycles(C.c_int(n), C.c_int(maxlvl), D(nu), C.c_int(cycles),
                               C.c_int(nthreads), C.byref(setup), C.byref(res))
    return t, setup.value, res.value
