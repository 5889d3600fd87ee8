"""Solver-level mirror of the reference's multigrid.cpp on the MI355X path.

* ``init_problem(N)``  -- multigrid.cpp:206-233 (host, glibc libm, bitwise inputs)
* ``timestepper(...)`` -- multigrid.cpp:124-186, same signature; host numpy arrays
* ``Multigrid``        -- the level towers resident in HBM (multigrid.cpp:131-162)
  with ``mg_inner()`` (multigrid.cpp:17-92, one V/W-cycle), ``mg_outer()``
  (multigrid.cpp:97-120), ``step()`` (one timestep, :165-172) and the op-level
  pieces ``gs``, ``residual_norm``, ``restrict``, ``prolong_add``, ``rhs``.

All compute runs in libmgx.so on the GPU; this module only marshals arguments.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib
from ._lib import check, default_options, lib


def _np_ptr(a: np.ndarray):
    if a.dtype != np.float64 or not a.flags["C_CONTIGUOUS"]:
        raise ValueError("expected a C-contiguous float64 array")
    return a.ctypes.data


def default_maxlvl(N: int) -> int:
    """multigrid.cpp:193: int(log2(N)) - 4 (coarsest n = 16... solved by GS)."""
    return int(math.log2(N)) - 4


def init_problem(N: int, nthreads: int = 0):
    """multigrid.cpp:206-233 -> (u0, v1, v2), each (N+1)^2 float64."""
    cnt = (N + 1) * (N + 1)
    u0, v1, v2 = (np.empty(cnt, dtype=np.float64) for _ in range(3))
    check(lib().mgx_init_problem(_np_ptr(u0), _np_ptr(v1), _np_ptr(v2), N, nthreads))
    return u0, v1, v2


def init_problem_rows(N: int, r0: int, r1: int, nthreads: int = 0):
    """Rows [r0, r1) of init_problem(N): three (r1-r0)*(N+1) float64 arrays."""
    cnt = (r1 - r0) * (N + 1)
    u0, v1, v2 = (np.empty(cnt, dtype=np.float64) for _ in range(3))
    check(lib().mgx_init_problem_rows(_np_ptr(u0), _np_ptr(v1), _np_ptr(v2), N, r0, r1,
                                      nthreads))
    return u0, v1, v2


def timestepper(uT, u0, v1, v2, nu, maxlvl, n, dt, T, dx, tol, shape=1, *, nsmooth=3,
                tower_mode=_lib.TOWER_REFERENCE, device=-1, fp_mode=_lib.FP_BITWISE):
    """multigrid.cpp:124 -- run (int)(T/dt) CN steps; writes uT, returns cycles per step."""
    steps = int(T / dt)
    cyc = (C.c_int * max(steps, 1))()
    opt = default_options(shape=shape, nsmooth=nsmooth, tower_mode=tower_mode, device=device,
                          fp_mode=fp_mode)
    check(lib().mgx_timestepper_ex(_np_ptr(uT), _np_ptr(u0), _np_ptr(v1), _np_ptr(v2), nu,
                                   maxlvl, n, dt, T, dx, tol, C.byref(opt), cyc))
    return list(cyc)[:steps]


def write_uT(path, rows, N: int, r0: int = 0, r1: int = None, append=False, nthreads=0):
    """multigrid.cpp:269-284 text output ("%d\t%d\t%f\n", i outer, j inner) of
    rows [r0, r1) held in `rows`; rank-ordered appends of row blocks give the
    whole-grid file byte for byte."""
    r1 = N + 1 if r1 is None else r1
    if rows.size != (r1 - r0) * (N + 1):
        raise ValueError("rows must hold (r1-r0)*(N+1) doubles")
    check(lib().mgx_write_uT(str(path).encode(), _np_ptr(rows), N, r0, r1, int(bool(append)),
                             nthreads))


class Multigrid:
    """Device-resident level towers and the V-cycle (mgx_ctx).

    Row-partitioned multi-GPU: ``world > 1`` with ``rank`` and the
    ``unique_id`` from ``dist.unique_id()`` (one process per GPU, RCCL), or
    ``local_parts=G`` for G virtual ranks on this GPU.  A partitioned solver
    takes the whole-solver calls (upload/download of the full grid, rhs,
    mg_inner, mg_outer, step, run_cycles, residual_norm(0)).
    """

    def __init__(self, N, maxlvl, dt, nu, *, nsmooth=3, shape=1,
                 tower_mode=_lib.TOWER_REFERENCE, device=-1, smoother=0, fuse=3,
                 coarse_tol=1e-5, coarse_maxit=1000, max_cycle=50,
                 world=1, rank=0, unique_id=None, local_parts=0, fp_mode=_lib.FP_BITWISE):
        self.N, self.maxlvl, self.dt, self.nu = N, maxlvl, dt, nu
        self.opt = default_options(nsmooth=nsmooth, shape=shape, tower_mode=tower_mode,
                                   device=device, smoother=smoother, fuse=fuse,
                                   coarse_tol=coarse_tol,
                                   coarse_maxit=coarse_maxit, max_cycle=max_cycle,
                                   fp_mode=fp_mode)
        h = C.c_void_p()
        if local_parts:
            check(lib().mgx_create_local_dist(C.byref(h), N, maxlvl, dt, nu,
                                              C.byref(self.opt), local_parts))
        elif world > 1 or unique_id is not None:
            if unique_id is None or len(unique_id) != _lib.UNIQUE_ID_BYTES:
                raise ValueError("world > 1 needs the 128-byte unique_id from rank 0")
            idbuf = C.create_string_buffer(bytes(unique_id), _lib.UNIQUE_ID_BYTES)
            check(lib().mgx_create_dist(C.byref(h), N, maxlvl, dt, nu, C.byref(self.opt),
                                        rank, world, idbuf))
        else:
            check(lib().mgx_create(C.byref(h), N, maxlvl, dt, nu, C.byref(self.opt)))
        self._h = h

    def dist_info(self):
        """-> (world, rank, first replicated level); rank -1 for local parts."""
        w, r, la = C.c_int(), C.c_int(), C.c_int()
        check(lib().mgx_dist_info(self._h, C.byref(w), C.byref(r), C.byref(la)))
        return w.value, r.value, la.value

    # -- lifetime
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().mgx_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # -- data
    def upload(self, u0, v1, v2):
        if isinstance(u0, np.ndarray):
            check(lib().mgx_upload(self._h, _np_ptr(u0), _np_ptr(v1), _np_ptr(v2)))
        else:   # device tensors in the reference layout
            check(lib().mgx_upload_device(self._h, u0.data_ptr(), v1.data_ptr(),
                                          v2.data_ptr()))

    def dist_rows(self, part=0):
        """-> (lo, hi): allocated finest-level rows of local part `part`."""
        lo, hi = C.c_int(), C.c_int()
        check(lib().mgx_dist_rows(self._h, part, C.byref(lo), C.byref(hi)))
        return lo.value, hi.value

    def upload_rows(self, blocks):
        """Row-block upload: blocks[i] = (u0, v1, v2) rows [lo, hi] of local part i
        (init_problem_rows); needs tower_mode=TOWER_CORRECT."""
        k = len(blocks)
        arr = C.c_void_p * k
        u, a, b = (arr(*[_np_ptr(blk[j]) for blk in blocks]) for j in range(3))
        check(lib().mgx_upload_rows(self._h, u, a, b))

    def owned_rows(self, part=0):
        """-> (ra, rb): finest-level rows [ra, rb) owned by local part `part`."""
        ra, rb = C.c_int(), C.c_int()
        check(lib().mgx_owned_rows(self._h, part, C.byref(ra), C.byref(rb)))
        return ra.value, rb.value

    def download_rows(self, part=0, out=None):
        """Row-block download: the owned rows of local part `part`,
        (rb-ra)*(N+1) float64 (no rank ever holds the whole grid)."""
        ra, rb = self.owned_rows(part)
        cnt = (rb - ra) * (self.N + 1)
        out = np.empty(cnt, dtype=np.float64) if out is None else out
        if out.size != cnt:
            raise ValueError(f"out must hold {cnt} doubles")
        check(lib().mgx_download_rows(self._h, part, _np_ptr(out)))
        return out

    def download(self, out=None):
        out = np.empty((self.N + 1) ** 2, dtype=np.float64) if out is None else out
        check(lib().mgx_download(self._h, _np_ptr(out)))
        return out

    def level_n(self, level):
        n = C.c_long()
        check(lib().mgx_level_n(self._h, level, C.byref(n)))
        return n.value

    def download_level(self, level, field="u"):
        f = {"u": 0, "rhs": 1, "v1": 2, "v2": 3}[field]
        n = self.level_n(level)
        out = np.empty((n + 1) ** 2, dtype=np.float64)
        check(lib().mgx_download_level(self._h, level, f, _np_ptr(out)))
        return out

    # -- ops (multigrid.cpp call sites)
    def rhs(self):
        check(lib().mgx_rhs(self._h))

    def gs(self, level, sweeps=1):
        check(lib().mgx_gs(self._h, level, sweeps))

    def residual_norm(self, level=0):
        r = C.c_double()
        check(lib().mgx_residual_norm(self._h, level, C.byref(r)))
        return r.value

    def restrict(self, level):
        check(lib().mgx_restrict(self._h, level))

    def prolong_add(self, level):
        check(lib().mgx_prolong_add(self._h, level))

    def mg_inner(self):
        """multigrid.cpp:17 at lvl=0: one V (shape=1) or W (shape=2) cycle."""
        check(lib().mgx_vcycle(self._h))

    vcycle = mg_inner

    def mg_outer(self, tol=1e-6):
        """multigrid.cpp:97 -> (cycles, res0, res); cap hit is reported, not raised."""
        cyc, r0, r = C.c_int(), C.c_double(), C.c_double()
        rc = check(lib().mgx_mg_outer(self._h, tol, C.byref(cyc), C.byref(r0), C.byref(r)),
                   allow=(_lib.MGX_E_NOCONV,))
        return cyc.value, r0.value, r.value, rc == _lib.MGX_E_NOCONV

    def step(self, tol=1e-6):
        cyc = C.c_int()
        check(lib().mgx_step(self._h, tol, C.byref(cyc)), allow=(_lib.MGX_E_NOCONV,))
        return cyc.value

    def run_cycles(self, cycles):
        r = C.c_double()
        check(lib().mgx_run_cycles(self._h, cycles, C.byref(r)))
        return r.value

    def coarse_iterations(self):
        it = C.c_long()
        check(lib().mgx_coarse_iterations(self._h, C.byref(it)))
        return it.value

    def synchronize(self):
        check(lib().mgx_synchronize(self._h))

    def stream(self):
        s = C.c_void_p()
        check(lib().mgx_stream(self._h, C.byref(s)))
        return s.value

    # -- profiling (HIP events on the context stream)
    def profile(self, on=True, finest_only=False):
        """HIP events around launches: all levels, or the finest level only."""
        check(lib().mgx_profile_enable(self._h, (2 if finest_only else 1) if on else 0))

    def profile_reset(self):
        check(lib().mgx_profile_reset(self._h))

    def profile_get(self, kind, level=-1):
        n, ms, b = C.c_long(), C.c_double(), C.c_double()
        check(lib().mgx_profile_get(self._h, kind, level, C.byref(n), C.byref(ms), C.byref(b)))
        return n.value, ms.value, b.value

    def profile_get_ex(self, kind, level=-1):
        """(launches, device ms, canonical algorithmic bytes, compulsory bytes)"""
        n, ms, b, cb = C.c_long(), C.c_double(), C.c_double(), C.c_double()
        check(lib().mgx_profile_get_ex(self._h, kind, level, C.byref(n), C.byref(ms),
                                       C.byref(b), C.byref(cb)))
        return n.value, ms.value, b.value, cb.value
