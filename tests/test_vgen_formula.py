"""CPU: the index map of the reference-tower velocity generator (stencil.h
vgen_rc, kernels.h VGen) against the CPU checker's reference tower
(oracle/mg_oracle.c or_build_tower, multigrid.cpp:148-160): level l's entry
(i, j) is the finest field's entry (I, I + 2J) after l injection steps of
next_s[m] -> next_{s-1}[I(N+2) + 2J], I, J = divmod(m, N/4+1), zero past
(N/4+1)^2 -- bit for bit on levels 1-3; and on levels 1-2 its closed form
(kernels.h VGen): a[2^l i + q] * b[2^l j - q(2W-1)], q = floor(2^(l-1)(j-i)/W),
zero where the flat index i(2W-1)+j (l = 1) / i(N+2)+2j (l = 2) reaches W^2."""
import numpy as np
import pytest

from oracle import oracle as O


def _gen(N, l, i, j, V):
    nl = N >> l
    W = N // 4 + 1
    if j > nl:
        return 0.0
    m = i * (nl + 1) + j
    for s in range(l):
        if m >= W * W:
            return 0.0
        I, J = divmod(m, W)
        if s + 1 == l:
            assert I + 2 * J < N + 1   # no carry into the next finest row
            return V[I, I + 2 * J]
        m = I * (N + 2) + 2 * J
    return None


@pytest.mark.parametrize("N", [64, 256])
def test_generator_reproduces_reference_tower(N):
    L = int(np.log2(N)) - 2
    u0, v1, v2 = O.init_problem(N)
    T = O.Tower(u0, v1, v2, N, L)
    try:
        for l in range(1, min(L, 4)):
            nl = N >> l
            for name, v in (("v1", v1), ("v2", v2)):
                V = v.reshape(N + 1, N + 1)
                got = np.array([[_gen(N, l, i, j, V) for j in range(nl + 1)]
                                for i in range(nl + 1)])
                ref = T.level(name, l).reshape(nl + 1, nl + 1)
                assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), (N, l, name)
                assert np.count_nonzero(ref) > 0
    finally:
        T.close()


def _closed(N, l, i, j, V):
    W = N // 4 + 1
    nl = N >> l
    m = i * (2 * W - 1) + j if l == 1 else i * (N + 2) + 2 * j
    if j > nl or m >= W * W:
        return 0.0
    d = (j - i) << (l - 1)
    q = -1 if d < 0 else (1 if d >= W else 0)
    return V[(i << l) + q, (j << l) - q * (2 * W - 1)]


@pytest.mark.parametrize("N", [64, 256, 1024])
def test_closed_form_levels_1_2(N):
    L = int(np.log2(N)) - 2
    u0, v1, v2 = O.init_problem(N)
    T = O.Tower(u0, v1, v2, N, L)
    try:
        for l in (1, 2):
            nl = N >> l
            for name, v in (("v1", v1), ("v2", v2)):
                V = v.reshape(N + 1, N + 1)
                got = np.array([[_closed(N, l, i, j, V) for j in range(nl + 1)]
                                for i in range(nl + 1)])
                ref = T.level(name, l).reshape(nl + 1, nl + 1)
                assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), (N, l, name)
    finally:
        T.close()
