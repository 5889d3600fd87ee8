"""Exact rank-1 velocity factors (csrc/sepvel.h, host code: no GPU).

The reference's rotating flow, v1 = -ky*sin(kx*i*dx)*cos(ky*j*dx) evaluated
left to right (/root/reference/multigrid.cpp:221-222), is fl(a_i * b_j)
exactly, so the finest cross pass may read two numbers per row instead of two
2-D rows.  The factorisation must reproduce EVERY entry bitwise or refuse:
random fields and rank-2 flows are refused, signed zeros count, and values
that would leave the normal range under the level scalings are refused.
"""
import ctypes as C

import numpy as np
import pytest

from hpcclassmultigridproject_amd import _lib, init_problem


def factor(v, N, smin=0.0):
    rows = v.size // (N + 1)
    a = np.empty(rows)
    b = np.empty(N + 1)
    r = _lib.lib().mgx_factor_velocity(v.ctypes.data, rows, N, smin, a.ctypes.data, b.ctypes.data)
    assert r in (0, 1), _lib.lib().mgx_last_error()
    return bool(r), a, b


@pytest.mark.parametrize("N", [32, 64, 1024, 4096])
def test_reference_flow_is_exactly_rank1(N):
    _, v1, v2 = init_problem(N)
    for v in (v1, v2):
        ok, a, b = factor(v, N, smin=0.5 / N)
        assert ok
        prod = np.multiply.outer(a, b).ravel()
        assert np.array_equal(prod.view(np.uint64), v.view(np.uint64))


def test_row_blocks_factor_on_their_own():
    """upload_rows: each rank factors only its rows (row 0 of v1 is all zeros)."""
    N = 1024
    _, v1, v2 = init_problem(N)
    W = N + 1
    for r0, r1 in ((0, 136), (120, 264), (888, W)):
        for v in (v1, v2):
            blk = v[r0 * W:r1 * W].copy()
            ok, a, b = factor(blk, N, smin=0.5 / N)
            assert ok
            assert np.array_equal(np.multiply.outer(a, b).ravel().view(np.uint64),
                                  blk.view(np.uint64))


def test_non_separable_fields_are_refused():
    N = 64
    rng = np.random.default_rng(20220501)
    assert not factor(rng.uniform(-1, 1, (N + 1) ** 2), N)[0]
    x = np.arange(N + 1) / N
    rank2 = (np.multiply.outer(np.sin(x), np.cos(x)) + np.multiply.outer(np.cos(x), x)).ravel()
    assert not factor(rank2, N)[0]
    # one flipped bit anywhere breaks it
    _, v1, _ = init_problem(N)
    w = v1.copy()
    w.view(np.uint64)[37 * (N + 1) + 11] ^= 1
    assert not factor(w, N)[0]
    # a signed zero in the wrong place breaks it too
    w = v1.copy()
    k = int(np.flatnonzero(w == 0)[0])
    w[k] = -w[k]
    assert not factor(w, N)[0] or np.array_equal(w.view(np.uint64), v1.view(np.uint64))


def test_scaling_range_is_checked():
    N = 16
    a = np.full(N + 1, 1e-300)
    b = np.linspace(1.0, 2.0, N + 1)
    v = np.multiply.outer(a, b).ravel()
    assert factor(v, N)[0]                       # exact product
    assert not factor(v, N, smin=1e-12)[0]       # but t = v*h/2 would be subnormal
