"""CPU checker (oracle/) against the reference's golden vectors and known answers.

The golden fixtures were produced by the unmodified reference sources
(tests/golden/make_golden.py); these tests pin the restatement to them
bitwise.  When the compiled reference (oracle/_ref) is present, the
restatement is also compared with it directly on fresh random cases.
"""
import math

import numpy as np
import pytest
from conftest import load_golden

NU = -4e-4


@pytest.mark.parametrize("N", [8, 16, 32, 64])
def test_ops_match_reference_fixture(oracle_mod, N):
    O = oracle_mod
    g = load_golden(f"ops_N{N}.npz")
    _, k, nu, h = g["params"]
    u, rhs, v1, v2 = g["u"], g["rhs"], g["v1"], g["v2"]
    gs = O.gauss_seidel(u.copy(), rhs, N, v1, v2, k, nu, h)
    assert np.array_equal(gs, g["gs"])
    res = O.residual(u, rhs, N, v1, v2, k, nu, h)
    assert np.array_equal(res, g["res"])
    assert O.compute_norm(res, N) == g["norm"][0]
    assert np.array_equal(O.compute_rhs(u, N, v1, v2, k, nu, h), g["crhs"])
    assert np.array_equal(O.prolongation(u, N), g["prol"])
    assert np.array_equal(O.restriction(u, N), g["restr"])


@pytest.mark.parametrize("tag", ["N32", "N64", "N128", "N128_nu001"])
def test_timestepper_matches_reference_fixture(oracle_mod, tag):
    O = oracle_mod
    g = load_golden(f"e2e_{tag}.npz")
    N, maxlvl, nu, dt, T, tol = g["params"]
    N, maxlvl = int(N), int(maxlvl)
    u0, v1, v2 = O.init_problem(N)
    uT, cyc = O.timestepper(u0, v1, v2, nu, maxlvl, N, dt, T, 1.0 / N, tol)
    assert np.array_equal(uT, g["uT"])
    assert cyc == list(g["cycles"])


def test_vcycle_matches_reference_fixture(oracle_mod):
    O = oracle_mod
    g = load_golden("vcycle_N256_L4.npz")
    N, maxlvl, nu, dt = g["params"]
    N, maxlvl = int(N), int(maxlvl)
    u0, v1, v2 = O.init_problem(N)
    t = O.Tower(u0, v1, v2, N, maxlvl)
    O.compute_rhs(t.ufine, N, v1, v2, dt, nu, 1.0 / N, rhs=t.rhsfine)
    t.mg_inner(dt, nu)
    assert np.array_equal(t.ufine, g["u"])


def test_vcycle_larger_matches_reference_summary(oracle_mod, golden_summary):
    import hashlib
    O = oracle_mod
    O.set_threads(4)
    try:
        # (N4096_L7_correct: the correct velocity tower, built by the
        # reference's own restriction at every level's true size)
        for tag in ("N1024_L6", "N4096_L3", "N4096_L7_correct"):
            s = golden_summary["vcycle"][tag]
            N, maxlvl = s["N"], s["maxlvl"]
            u0, v1, v2 = O.init_problem(N)
            dt = 1.0 / N / 10
            t = O.Tower(u0, v1, v2, N, maxlvl, 1 if s.get("tower") == "correct" else 0)
            O.compute_rhs(t.ufine, N, v1, v2, dt, NU, 1.0 / N, rhs=t.rhsfine)
            t.mg_inner(dt, NU)
            assert hashlib.sha256(t.ufine.tobytes()).hexdigest() == s["sha256"], tag
            t.close()
    finally:
        O.set_threads(1)


def test_threads_equal_serial(oracle_mod):
    """multigrid.cpp:261-266: the threaded run equals the serial one (K1)."""
    O = oracle_mod
    N = 128
    u0, v1, v2 = O.init_problem(N)
    dx = 1.0 / N
    ref, _ = O.timestepper(u0, v1, v2, NU, 3, N, dx / 10, 10 * dx / 10, dx)
    O.set_threads(4)
    try:
        par, _ = O.timestepper(u0, v1, v2, NU, 3, N, dx / 10, 10 * dx / 10, dx)
    finally:
        O.set_threads(1)
    assert np.array_equal(ref, par)


def test_prolongation_restriction_kat(oracle_mod):
    """prolrestest.cpp:64-118: u=i+j, prolongation exact, restriction recovers it."""
    O = oracle_mod
    N = 5
    i, j = np.meshgrid(np.arange(N + 1), np.arange(N + 1), indexing="ij")
    u = (i + j).astype(np.float64).ravel()
    up = O.prolongation(u, N)
    I, J = np.meshgrid(np.arange(2 * N + 1), np.arange(2 * N + 1), indexing="ij")
    assert np.array_equal(up, ((I + J) / 2.0).ravel())
    back = np.zeros_like(u)
    m = 2 * N // 2 + 1
    back = O.restriction(up, 2 * N)
    assert np.array_equal(back, u[: m * m])


def test_gs_black_residual_vanishes(oracle_mod):
    """After a sweep the last-updated colour (black) has ~zero residual."""
    O = oracle_mod
    g = load_golden("ops_N32.npz")
    N, k, nu, h = g["params"]
    N = int(N)
    u = O.gauss_seidel(g["u"].copy(), g["rhs"], N, g["v1"], g["v2"], k, nu, h)
    r = O.residual(u, g["rhs"], N, g["v1"], g["v2"], k, nu, h).reshape(N + 1, N + 1)
    ii, jj = np.meshgrid(np.arange(N + 1), np.arange(N + 1), indexing="ij")
    black = ((ii + jj) % 2 == 1) & (ii > 0) & (ii < N) & (jj > 0) & (jj < N)
    assert np.abs(r[black]).max() < 1e-14
    assert np.abs(r[~black & (ii > 0) & (ii < N) & (jj > 0) & (jj < N)]).max() > 1e-6


def test_correct_tower_is_close_to_reference_tower(oracle_mod):
    """the correctly injected tower changes uT by <= ~1e-15."""
    O = oracle_mod
    N = 128
    u0, v1, v2 = O.init_problem(N)
    dx = 1.0 / N
    a, ca = O.timestepper(u0, v1, v2, NU, 3, N, dx / 10, 100 * dx / 10, dx, tower_mode=0)
    b, cb = O.timestepper(u0, v1, v2, NU, 3, N, dx / 10, 100 * dx / 10, dx, tower_mode=1)
    assert ca == cb
    assert np.abs(a - b).max() <= 1e-12


@pytest.fixture(scope="module")
def ref_lib(oracle_mod):
    if not oracle_mod.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    return oracle_mod.ref()


@pytest.mark.parametrize("N,shape", [(64, 1), (64, 2), (128, 2)])
def test_restatement_equals_reference_timestepper(oracle_mod, ref_lib, N, shape):
    O = oracle_mod
    maxlvl = int(math.log2(N)) - 4
    u0, v1, v2 = O.init_problem(N)
    dx = 1.0 / N
    dt = dx / 10
    a = O.ref_timestepper(u0, v1, v2, NU, maxlvl, N, dt, 20 * dt, dx, 1e-6, shape)
    b, _ = O.timestepper(u0, v1, v2, NU, maxlvl, N, dt, 20 * dt, dx, shape=shape)
    assert np.array_equal(a, b)


def test_restatement_equals_reference_ops_random(oracle_mod, ref_lib):
    import ctypes as C
    O = oracle_mod
    rng = np.random.default_rng(7)
    P = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    for N in (6, 10, 40):
        cnt = (N + 1) ** 2
        u, rhs, v1, v2 = (rng.uniform(-3, 3, cnt) for _ in range(4))
        k, nu, h = 0.37 / N, -0.013, 1.0 / N
        a = u.copy()
        ref_lib.ref_gauss_seidel(P(a), P(rhs), C.c_long(N), P(v1), P(v2), C.c_double(k),
                                 C.c_double(nu), C.c_double(h), C.c_int(1))
        assert np.array_equal(a, O.gauss_seidel(u.copy(), rhs, N, v1, v2, k, nu, h))


@pytest.mark.parametrize("N,maxlvl", [(128, 3), (256, 4)])
def test_restatement_equals_reference_nu2(oracle_mod, N, maxlvl):
    """Config 2's smoothing count (2 pre/post sweeps) against the reference
    built with NITER=2 (oracle/Makefile libmgref_nu2.so): 20 timesteps bitwise."""
    O = oracle_mod
    if not O.ref_available(2):
        pytest.skip("oracle/_ref/libmgref_nu2.so not built")
    u0, v1, v2 = O.init_problem(N)
    dx = 1.0 / N
    dt = dx / 10
    uT_ref = O.ref_timestepper(u0, v1, v2, -4e-4, maxlvl, N, dt, 20 * dt, dx, nsmooth=2)
    uT, cyc = O.timestepper(u0, v1, v2, -4e-4, maxlvl, N, dt, 20 * dt, dx, nsmooth=2)
    assert np.array_equal(uT, uT_ref)
    # NITER really is 2 there: the unmodified reference gives a different answer
    assert not np.array_equal(uT, O.ref_timestepper(u0, v1, v2, -4e-4, maxlvl, N, dt,
                                                     20 * dt, dx))


def test_config2_summary_from_nu2_reference(golden_summary):
    s = golden_summary["steps"]["N4096_L3_nu2_2steps"]
    assert s["nsmooth"] == 2 and s["cycles"] == [2, 2]   # C2, 2 cycles/step


@pytest.mark.parametrize("N,r0,nr", [(64, 0, 12), (64, 20, 9), (64, 55, 10), (64, 0, 65),
                                     (33, 17, 17)])
def test_slab_ops_equal_whole_field(oracle_mod, N, r0, nr):
    """The row-slab forms (the N=65536 GPU checks' oracle) are the whole-field
    ops on the rows their window determines, seeded random fields."""
    O = oracle_mod
    rng = np.random.default_rng(20220501)
    w = N + 1
    u, rhs = rng.uniform(-1, 1, w * w), rng.uniform(-1, 1, w * w)
    v1, v2 = rng.uniform(-3, 3, w * w), rng.uniform(-3, 3, w * w)
    k, h = 1.0 / N / 10, 1.0 / N
    sl = slice(r0 * w, (r0 + nr) * w)
    full = O.gauss_seidel(u.copy(), rhs, N, v1, v2, k, NU, h)
    slab = O.gauss_seidel_slab(u[sl].copy(), rhs[sl], N, r0, v1[sl], v2[sl], k, NU, h)
    a, b = (r0 + 2 if r0 > 0 else 0), min(N + 1, r0 + nr - 2 if r0 + nr <= N else N + 1)
    assert np.array_equal(slab[(a - r0) * w:(b - r0) * w], full[a * w:b * w])
    res_f = O.residual(u, rhs, N, v1, v2, k, NU, h)
    res_s = O.residual_slab(u[sl].copy(), rhs[sl], N, r0, v1[sl], v2[sl], k, NU, h)
    a1, b1 = max(1, r0 + 1), min(N, r0 + nr - 1)
    assert np.array_equal(res_s[(a1 - r0) * w:(b1 - r0) * w], res_f[a1 * w:b1 * w])
    crhs_f = O.compute_rhs(u, N, v1, v2, k, NU, h)
    crhs_s = O.compute_rhs_slab(u[sl].copy(), N, r0, v1[sl], v2[sl], k, NU, h)
    assert np.array_equal(crhs_s[(a1 - r0) * w:(b1 - r0) * w], crhs_f[a1 * w:b1 * w])
    W = 2 * N + 1
    pf = O.prolongation(u, N)
    ps = O.prolongation_slab(u[sl].copy(), N, r0)
    I1 = min(2 * (r0 + nr - 1), 2 * N)
    assert np.array_equal(ps, pf[2 * r0 * W:(I1 + 1) * W])


@pytest.mark.parametrize("tag", ["N32", "N64", "N128", "N128_nu001"])
def test_fma_form_within_tolerance_of_reference(oracle_mod, tag):
    """The checker's restatement of libmgx's fp_mode fma (or_set_fp_mode)
    against the reference's own 100-step uT: max|duT| <= 1e-12 with the same
    cycle counts -- the contracted form meets the stated
    tolerance on the CPU as well; on the GPU the fma kernels equal this
    restatement bit for bit (tests/test_gpu_fma.py)."""
    O = oracle_mod
    g = load_golden(f"e2e_{tag}.npz")
    N, maxlvl, nu, dt, T, tol = g["params"]
    N, maxlvl = int(N), int(maxlvl)
    u0, v1, v2 = O.init_problem(N)
    O.set_fp_mode(1)
    try:
        uT, cyc = O.timestepper(u0, v1, v2, nu, maxlvl, N, dt, T, 1.0 / N, tol)
    finally:
        O.set_fp_mode(0)
    assert cyc == list(g["cycles"])
    err = float(np.max(np.abs(uT - g["uT"])))
    assert 0 < err <= 1e-12, err
