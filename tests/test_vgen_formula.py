"""CPU: the closed form behind level 1's velocity generator (stencil.h
vg_col / vg_state / vg_row, kernels.h VGen) against the CPU checker's
reference tower (oracle/mg_oracle.c or_build_tower, multigrid.cpp:148-160).

Level 1 of the reference tower reads the finest field through the injection's
index quirk: entry (i, j) is the finest entry (2i + q, 2j -
q(2W-1)), q = floor((j-i)/W), W = N/4 + 1, while i(2W-1) + j < W^2, zero
beyond.  The kernel walks each column down the rows with three states (q =
qh, q = qh - 1, zero); this test evaluates exactly those integer expressions
and checks every entry of both fields bit for bit."""
import numpy as np
import pytest

from oracle import oracle as O


def vg_col(j, n):
    W, den, N = n // 2 + 1, n + 1, 2 * n
    assert den == 2 * W - 1
    if j < 0 or j > n:
        return 0, 0, -0x7fffffff, 0, 0
    qh = j // W
    rt = j - qh * W + 1
    rz = (W * W - j + den - 1) // den
    chi, clo = 2 * j - qh * den, 2 * j - qh * den + den
    return qh, rt, rz, min(max(chi, 0), N), min(max(clo, 0), N)


def vg_value(i, j, n, A):
    qh, rt, rz, chi, clo = vg_col(j, n)
    st = 2 if i >= rz else (1 if i >= rt else 0)
    if st == 2:
        return 0.0
    I, c = 2 * i + qh - st, (clo if st == 1 else chi)
    assert 0 <= I <= 2 * n and 0 <= c <= 2 * n
    return A[I, c]


@pytest.mark.parametrize("N", [64, 256])
def test_level1_closed_form_reproduces_reference_tower(N):
    L = int(np.log2(N)) - 2
    u0, v1, v2 = O.init_problem(N)
    T = O.Tower(u0, v1, v2, N, L)
    try:
        n = N // 2
        for name, v in (("v1", v1), ("v2", v2)):
            V = v.reshape(N + 1, N + 1)
            got = np.array([[vg_value(i, j, n, V) for j in range(n + 1)]
                            for i in range(n + 1)])
            ref = T.level(name, 1).reshape(n + 1, n + 1)
            assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), (N, name)
            nz = np.count_nonzero(ref, axis=1)
            assert nz[0] > 0 and nz[-1] == 0   # zero rows exist: the third state is exercised
    finally:
        T.close()


@pytest.mark.parametrize("N", [64, 256, 1024, 16384, 32768])
def test_each_column_has_at_most_one_q_step_before_its_zero_rows(N):
    """The premise of the per-column states: over the nonzero rows i < rz the
    quotient q = floor((j-i)/W) takes at most two values, qh and qh - 1."""
    n = N // 2
    W = n // 2 + 1
    for j in range(0, n + 1, max(1, n // 257)):
        qh, rt, rz, chi, clo = vg_col(j, n)
        qs = {(j - i) // W for i in range(0, min(rz, n + 1))}
        assert qs <= {qh, qh - 1}, (N, j, qs)
        for i in range(0, min(rz, n + 1)):
            assert (j - i) // W == (qh if i < rt else qh - 1)
            assert i * (2 * W - 1) + j < W * W
        if rz <= n:
            assert rz * (2 * W - 1) + j >= W * W
