"""The generated coarse velocity (tuning key "vgen", kernels.h VGen, stencil.h
vg_col): the V-cycle's 3-sweep pre / post marches of levels 1-2 of the
reference tower, and of every level below the coarsest of the correct tower
(v_l(i, j) = fl(a[2^l i] * b[2^l j]), /root/reference/multigrid.cpp:148-160 as
a correct injection, gs.cpp:268-292), regenerate v1, v2 from the finest
level's factors instead of reading them.  Enabled only when the upload check
finds every entry of the level equal to the generator's bits, so u, norms and
cycle counts must be BITWISE those of the read path, in both fp modes, for
V-cycles (with the cross-cycle pass), plain cycles and time steps -- on one
GPU, on row blocks of a whole-grid upload, and on row blocks of the row-block
upload (each rank's own factors, ghost rows' factors from its exchanged
rows)."""
import ctypes

import numpy as np
import pytest

from hpcclassmultigridproject_amd import Multigrid, _lib, init_problem

pytestmark = pytest.mark.gpu
NU = -4e-4


def _factored(mg):
    f = ctypes.c_int(0)
    _lib.check(_lib.lib().mgx_velocity_factored(mg.handle, ctypes.byref(f)))
    return f.value


def _run(N, L, fp, vgen, cycles=3, steps=2, tower=_lib.TOWER_REFERENCE, perturb=False):
    old = _lib.get_tuning("vgen")
    _lib.set_tuning("vgen", vgen)
    try:
        u0, v1, v2 = init_problem(N)
        if perturb:   # not rank-1 any more: no factors, no generator
            v1.reshape(-1)[N // 3 * (N + 1) + N // 5] *= 1.0000001
        with Multigrid(N, L, 1.0 / N / 10, NU, fp_mode=fp, tower_mode=tower) as mg:
            mg.upload(u0, v1, v2)
            fac = _factored(mg)
            mg.rhs()
            norms = [mg.run_cycles(1) for _ in range(cycles)]
            ua = mg.download(np.empty_like(u0))
            cyc = [mg.step(1e-6) for _ in range(steps)]
            ub = mg.download(np.empty_like(u0))
            return fac, norms, ua, cyc, ub
    finally:
        _lib.set_tuning("vgen", old)


@pytest.mark.parametrize("fp", [_lib.FP_BITWISE, _lib.FP_FMA], ids=["bitwise", "fma"])
@pytest.mark.parametrize("N,L", [(4096, 7), (16384, 9)])
def test_generated_coarse_velocity_bitwise_vs_read(N, L, fp):
    fa, na, ua, ca, ub = _run(N, L, fp, 1)
    fb, nb, va, cb, vb = _run(N, L, fp, 0)
    assert fa == 7, fa          # finest factors + levels 1, 2 generating
    assert fb == 1, fb
    assert na == nb
    assert np.array_equal(ua.view(np.uint64), va.view(np.uint64))
    assert ca == cb
    assert np.array_equal(ub.view(np.uint64), vb.view(np.uint64))


def test_no_generator_without_factors():
    # a non-rank-1 field has no factors, so no level generates
    assert _run(4096, 7, _lib.FP_FMA, 1, cycles=1, steps=0, perturb=True)[0] == 0
    assert _run(4096, 7, _lib.FP_FMA, 1, cycles=1, steps=0, perturb=True,
                tower=_lib.TOWER_CORRECT)[0] == 0


@pytest.mark.parametrize("fp", [_lib.FP_BITWISE, _lib.FP_FMA], ids=["bitwise", "fma"])
@pytest.mark.parametrize("N,L", [(4096, 7), (16384, 9)])
def test_generated_velocity_correct_tower_bitwise_vs_read(N, L, fp):
    """The correct tower: every level below the coarsest generates (strided
    factors), bitwise the read path."""
    fa, na, ua, ca, ub = _run(N, L, fp, 1, tower=_lib.TOWER_CORRECT)
    fb, nb, va, cb, vb = _run(N, L, fp, 0, tower=_lib.TOWER_CORRECT)
    assert fa == (1 << (L - 1)) - 1, bin(fa)   # finest factors + levels 1..L-2
    assert fb == 1, fb
    assert na == nb
    assert np.array_equal(ua.view(np.uint64), va.view(np.uint64))
    assert ca == cb
    assert np.array_equal(ub.view(np.uint64), vb.view(np.uint64))


def _rows_run(vgen, parts, N, L, fp=_lib.FP_FMA):
    """Row-block upload (the C5 path) on virtual ranks, correct tower."""
    from hpcclassmultigridproject_amd import init_problem_rows
    old = _lib.get_tuning("vgen")
    _lib.set_tuning("vgen", vgen)
    try:
        with Multigrid(N, L, 1.0 / N / 10, NU, fp_mode=fp, tower_mode=_lib.TOWER_CORRECT,
                       local_parts=parts) as mg:
            blocks = []
            for part in range(parts):
                lo, hi = mg.dist_rows(part)
                blocks.append(init_problem_rows(N, lo, hi + 1))
            mg.upload_rows(blocks)
            del blocks
            fac = _factored(mg)
            la = mg.dist_info()[2]
            mg.rhs()
            mg.profile(True)
            norms = [mg.run_cycles(1) for _ in range(3)]
            cb = [sum(mg.profile_get_ex(k, l)[3] for k in (_lib.K_GS, _lib.K_PSMOOTH))
                  for l in range(1, la)]
            mg.profile(False)
            u = mg.download()
            cyc = [mg.step(1e-6) for _ in range(2)]
            return fac, la, norms, u, cyc, mg.download(), cb
    finally:
        _lib.set_tuning("vgen", old)


@pytest.mark.parametrize("N,L,parts", [(4096, 7, 2), (16384, 9, 8)])
def test_generated_velocity_row_block_upload_bitwise(N, L, parts):
    """Row-block upload, 2 and 8 virtual ranks: every partitioned coarse
    level generates from its block's factors (ghost rows' factors filled from
    its exchanged rows), bitwise the read path and the one-GPU result."""
    fa, la, na, ua, ca, wa, cba = _rows_run(1, parts, N, L)
    fb, lb, nb, ub, cb, wb, cbb = _rows_run(0, parts, N, L)
    assert la == lb and la >= 2
    assert fa == (1 << la) - 1, (bin(fa), la)   # level 0's factors + levels 1..la-1
    assert fb == 1, fb
    assert na == nb and ca == cb
    assert np.array_equal(ua.view(np.uint64), ub.view(np.uint64))
    assert np.array_equal(wa.view(np.uint64), wb.view(np.uint64))
    # level 1 always marches, so its passes read two arrays less
    assert cba[0] < 0.8 * cbb[0], (cba, cbb)
    # and the one-GPU correct-tower solve, generated too: the same bits
    f1, n1, u1, c1, w1 = _run(N, L, _lib.FP_FMA, 1, tower=_lib.TOWER_CORRECT, cycles=3)
    assert np.array_equal(ua.view(np.uint64), u1.view(np.uint64))
    assert c1 == ca
    assert np.array_equal(wa.view(np.uint64), w1.view(np.uint64))
    np.testing.assert_allclose(na, n1, rtol=1e-11)


def _dist_run(vgen, parts, N=16384, L=9):
    old = _lib.get_tuning("vgen")
    _lib.set_tuning("vgen", vgen)
    try:
        u0, v1, v2 = init_problem(N)
        with Multigrid(N, L, 1.0 / N / 10, NU, fp_mode=_lib.FP_FMA, local_parts=parts) as mg:
            mg.upload(u0, v1, v2)
            mg.rhs()
            mg.profile(True)
            norms = [mg.run_cycles(1) for _ in range(3)]
            # compulsory bytes of levels 1-2's smoothing passes (launch accounting)
            cb = [sum(mg.profile_get_ex(k, l)[3] for k in (_lib.K_GS, _lib.K_PSMOOTH))
                  for l in (1, 2)]
            mg.profile(False)
            return norms, mg.download(np.empty_like(u0)), cb
    finally:
        _lib.set_tuning("vgen", old)


@pytest.mark.parametrize("parts", [2, 8])
def test_generated_velocity_on_row_blocks_bitwise(parts):
    """Virtual ranks (the row-block code path, dist.hip): levels 1-2's blocks
    generate their rows of the velocity from level 0's global factors --
    bitwise the read path, and the passes' compulsory bytes drop by the two
    velocity arrays."""
    na, ua, ca = _dist_run(1, parts)
    nb, ub, cb = _dist_run(0, parts)
    assert na == nb
    assert np.array_equal(ua.view(np.uint64), ub.view(np.uint64))
    # (level 1 always marches; level 2's blocks at 8 parts may run as LDS
    # tiles, which read the arrays)
    assert ca[0] < 0.75 * cb[0] and ca[1] <= cb[1], (ca, cb)
    if parts == 2:
        assert ca[1] < 0.75 * cb[1], (ca, cb)
