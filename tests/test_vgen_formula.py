"""CPU: the closed form behind the velocity generator of levels 1-2 (stencil.h
vg_col / vg_state / vg_row, kernels.h VGen) against the CPU checker's
reference tower (oracle/mg_oracle.c or_build_tower, multigrid.cpp:148-160).

Levels 1-2 of the reference tower read the finest field through the
injection's index quirk: with s = 2^(l-1), W = N/4 + 1, entry
(i, j) of level l is the finest entry (2s i + q, 2s j - q(2W-1)), q =
floor(s(j-i)/W), while s(i(2W-1) + j) < W^2, zero beyond.  The kernel walks
each column down the rows with three states (q = qh, q = qh - 1, zero); this
test evaluates exactly those integer expressions and checks every entry of
both fields bit for bit."""
import numpy as np
import pytest

from oracle import oracle as O


def vg_col(j, n, l):
    N = n << l
    W, s = N // 4 + 1, 1 << (l - 1)
    den = 2 * W - 1
    if j < 0 or j > n:
        return 0, 0, -0x7fffffff, 0, 0
    qh = s * j // W
    rt = (s * j - qh * W) // s + 1
    rz = (W * W - s * j + s * den - 1) // (s * den)
    chi = 2 * s * j - qh * den
    return qh, rt, rz, min(max(chi, 0), N), min(max(chi + den, 0), N)


def vg_value(i, j, n, l, V):
    qh, rt, rz, chi, clo = vg_col(j, n, l)
    st = 2 if i >= rz else (1 if i >= rt else 0)
    if st == 2:
        return 0.0
    I, c = (i << l) + qh - st, (clo if st == 1 else chi)
    assert 0 <= I <= n << l and 0 <= c <= n << l
    return V[I, c]


@pytest.mark.parametrize("N", [64, 256])
@pytest.mark.parametrize("l", [1, 2])
def test_closed_form_reproduces_reference_tower(N, l):
    L = int(np.log2(N)) - 2
    u0, v1, v2 = O.init_problem(N)
    T = O.Tower(u0, v1, v2, N, L)
    try:
        n = N >> l
        for name, v in (("v1", v1), ("v2", v2)):
            V = v.reshape(N + 1, N + 1)
            got = np.array([[vg_value(i, j, n, l, V) for j in range(n + 1)]
                            for i in range(n + 1)])
            ref = T.level(name, l).reshape(n + 1, n + 1)
            assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), (N, l, name)
            nz = np.count_nonzero(ref, axis=1)
            assert nz[0] > 0 and nz[-1] == 0   # zero rows exist: the third state is exercised
    finally:
        T.close()


@pytest.mark.parametrize("N", [64, 256, 1024, 16384, 32768])
@pytest.mark.parametrize("l", [1, 2])
def test_each_column_has_at_most_one_q_step_before_its_zero_rows(N, l):
    """The premise of the per-column states: over the nonzero rows i < rz the
    quotient q = floor(s(j-i)/W) takes at most two values, qh and qh - 1."""
    n = N >> l
    W, s = N // 4 + 1, 1 << (l - 1)
    for j in range(0, n + 1, max(1, n // 257)):
        qh, rt, rz, chi, clo = vg_col(j, n, l)
        rows = range(0, min(rz, n + 1))
        assert {s * (j - i) // W for i in rows} <= {qh, qh - 1}, (N, l, j)
        for i in rows:
            assert s * (j - i) // W == (qh if i < rt else qh - 1)
            assert s * (i * (2 * W - 1) + j) < W * W
        if rz <= n:
            assert s * (rz * (2 * W - 1) + j) >= W * W
