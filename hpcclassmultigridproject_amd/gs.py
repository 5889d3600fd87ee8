"""Op-level mirror of the reference's gs.h (gs.h:3-17, gs.cpp).

Same names, argument order and meaning as the reference; arrays are DEVICE
buffers in the reference layout (row-major (n+1)^2 float64): torch CUDA
tensors (PyTorch is used only as the device allocator) or raw device pointers
(int).  Each call is a HIP kernel in libmgx.so; there is no CPU path.

Like the reference, ``gauss_seidel`` updates ``u`` in place, ``residual`` and
``compute_rhs`` write only the interior of their output, ``compute_norm``
returns a Python float.  ``prolongation(up, u, n)`` writes (2n+1)^2 values,
``restriction(u, up, n)`` writes (n/2+1)^2 values (including the boundary).
"""
from __future__ import annotations

import ctypes as C

from ._lib import check, lib


def _ptr(x, count=None):
    if isinstance(x, int):
        return x
    # torch tensor
    if not x.is_cuda:
        raise ValueError("expected a device (cuda) tensor")
    if x.dtype != __import__("torch").float64:
        raise ValueError("expected float64")
    if not x.is_contiguous():
        raise ValueError("expected a contiguous tensor")
    if count is not None and x.numel() < count:
        raise ValueError(f"tensor has {x.numel()} elements, need {count}")
    return x.data_ptr()


def _m(n):
    return (n + 1) * (n + 1)


def gauss_seidel(u, rhs, n, v1, v2, k, nu, h):
    """gs.cpp:109-189 -- one red-black sweep, in place on u."""
    m = _m(n)
    check(lib().mgx_gauss_seidel(_ptr(u, m), _ptr(rhs, m), n, _ptr(v1, m), _ptr(v2, m),
                                 k, nu, h))


def residual(res, u, rhs, n, v1, v2, k, nu, h):
    """gs.cpp:55-83 -- res = rhs - A u on the interior (boundary of res untouched)."""
    m = _m(n)
    check(lib().mgx_residual(_ptr(res, m), _ptr(u, m), _ptr(rhs, m), n, _ptr(v1, m),
                             _ptr(v2, m), k, nu, h))


def compute_norm(res, n) -> float:
    """gs.cpp:86-107 -- sqrt of the sum of the interior squares."""
    out = C.c_double()
    check(lib().mgx_compute_norm(_ptr(res, _m(n)), n, C.byref(out)))
    return out.value


def prolongation(up, u, n):
    """gs.cpp:228-266 -- up ((2n+1)^2) = bilinear interpolation of u ((n+1)^2)."""
    check(lib().mgx_prolongation(_ptr(up, (2 * n + 1) ** 2), _ptr(u, _m(n)), n))


def restriction(u, up, n):
    """gs.cpp:268-292 -- u ((n/2+1)^2) = injection of up ((n+1)^2)."""
    check(lib().mgx_restriction(_ptr(u, (n // 2 + 1) ** 2), _ptr(up, _m(n)), n))


def compute_rhs(rhs, u, n, v1, v2, k, nu, h):
    """gs.cpp:24-53 -- Crank-Nicolson right-hand side on the interior."""
    m = _m(n)
    check(lib().mgx_compute_rhs(_ptr(rhs, m), _ptr(u, m), n, _ptr(v1, m), _ptr(v2, m),
                                k, nu, h))
