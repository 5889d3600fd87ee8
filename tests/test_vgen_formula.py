"""CPU: the index map of the reference-tower velocity generator (stencil.h
vgen_rc, kernels.h VGen) against the CPU checker's reference tower
(oracle/mg_oracle.c or_build_tower, multigrid.cpp:148-160): level l's entry
(i, j) is the finest field's entry (I, I + 2J) after l injection steps of
next_s[m] -> next_{s-1}[I(N+2) + 2J], I, J = divmod(m, N/4+1), zero past
(N/4+1)^2 -- bit for bit on levels 1-3."""
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
