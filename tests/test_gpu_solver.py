"""GPU parity of the solver level: V-cycle, mg_outer, timestepper.

Bar: the solution after any number of V-cycles / timesteps is BITWISE the
reference's (reference tower mode), checked against the golden fixtures made
by the reference itself, and against the CPU checker where no fixture exists
(nu_smooth=2, W-cycles, correct-tower mode).  Cycle counts must be identical.
"""
import hashlib
import math

import numpy as np
import pytest
from conftest import load_golden

from hpcclassmultigridproject_amd import Multigrid, _lib, init_problem, timestepper

pytestmark = pytest.mark.gpu
NU = -4e-4


@pytest.mark.parametrize("tag", ["N32", "N64", "N128", "N128_nu001"])
def test_timestepper_bitwise_vs_reference(tag):
    g = load_golden(f"e2e_{tag}.npz")
    N, maxlvl, nu, dt, T, tol = g["params"]
    N, maxlvl = int(N), int(maxlvl)
    u0, v1, v2 = init_problem(N)
    uT = np.empty_like(u0)
    cyc = timestepper(uT, u0, v1, v2, nu, maxlvl, N, dt, T, 1.0 / N, tol)
    assert cyc == list(g["cycles"])
    assert np.array_equal(uT, g["uT"])


@pytest.fixture(params=[2048, 0], ids=["tile", "march"])
def tile_mode(request):
    from hpcclassmultigridproject_amd import _lib
    old = _lib.get_tuning("tile_max_n")
    _lib.set_tuning("tile_max_n", request.param)
    yield request.param
    _lib.set_tuning("tile_max_n", old)


@pytest.mark.parametrize("smoother,fuse", [(0, 3), (0, 2), (0, 1), (1, 3), (2, 3)])
def test_vcycle_bitwise_vs_reference_N256(smoother, fuse, tile_mode):
    g = load_golden("vcycle_N256_L4.npz")
    N, maxlvl, nu, dt = g["params"]
    N, maxlvl = int(N), int(maxlvl)
    u0, v1, v2 = init_problem(N)
    with Multigrid(N, maxlvl, dt, nu, smoother=smoother, fuse=fuse) as mg:
        mg.upload(u0, v1, v2)
        mg.rhs()
        mg.mg_inner()
        assert np.array_equal(mg.download(), g["u"])


@pytest.mark.parametrize("tag", ["N1024_L6", "N4096_L3"])
def test_vcycle_bitwise_vs_reference_summary(golden_summary, tag):
    s = golden_summary["vcycle"][tag]
    N, maxlvl = s["N"], s["maxlvl"]
    u0, v1, v2 = init_problem(N)
    dt = 1.0 / N / 10
    with Multigrid(N, maxlvl, dt, NU) as mg:
        mg.upload(u0, v1, v2)
        mg.rhs()
        mg.mg_inner()
        u = mg.download()
        assert hashlib.sha256(u.tobytes()).hexdigest() == s["sha256"]
        r = mg.residual_norm(0)
        assert abs(r - float(s["res_after"])) <= 1e-11 * float(s["res_after"])


@pytest.mark.slow
def test_vcycle_bitwise_vs_reference_N16384(golden_summary):
    """Headline size (config 3): one V-cycle, L=9 (coarsest 64), nu_smooth=3."""
    s = golden_summary["vcycle"].get("N16384_L9")
    if s is None:
        pytest.skip("large fixture not generated")
    N, maxlvl = 16384, 9
    u0, v1, v2 = init_problem(N)
    dt = 1.0 / N / 10
    with Multigrid(N, maxlvl, dt, NU) as mg:
        mg.upload(u0, v1, v2)
        del v1, v2
        mg.rhs()
        mg.mg_inner()
        u = mg.download(u0)
        assert hashlib.sha256(u.tobytes()).hexdigest() == s["sha256"]
        g = load_golden("vcycle_N16384_L9.npz")
        step = N // 64
        assert np.array_equal(u.reshape(N + 1, N + 1)[::step, ::step], g["sample"])


@pytest.mark.parametrize("tag", ["N4096_L7_correct", "N16384_L9_correct"])
def test_vcycle_correct_tower_vs_reference(golden_summary, tag):
    """TOWER_CORRECT (every coarse velocity level injected from the one
    above at its true size; the tower every row-block and N > 16384 run uses)
    at the headline size: one V-cycle bitwise equal to the compiled
    reference's mg_inner on the same tower (sha256 and the 65x65 sample,
    tests/golden/make_golden.py correct_tower_fixtures); the fma mode within
    SURVEY K3's 1e-12 of it, same residual to 1e-9 relative."""
    s = golden_summary["vcycle"][tag]
    N, maxlvl = s["N"], s["maxlvl"]
    u0, v1, v2 = init_problem(N)
    dt = 1.0 / N / 10
    out = {}
    for fp in (_lib.FP_BITWISE, _lib.FP_FMA):
        with Multigrid(N, maxlvl, dt, NU, tower_mode=_lib.TOWER_CORRECT, fp_mode=fp) as mg:
            mg.upload(u0, v1, v2)
            mg.rhs()
            mg.mg_inner()
            out[fp] = (mg.download(), mg.residual_norm(0))
    ub, rb = out[_lib.FP_BITWISE]
    assert hashlib.sha256(ub.tobytes()).hexdigest() == s["sha256"]
    g = load_golden(f"vcycle_{tag}.npz")
    step = N // 64
    assert np.array_equal(ub.reshape(N + 1, N + 1)[::step, ::step], g["sample"])
    # the norm differs only by summation order: the reference sums (N-1)^2
    # squares serially (2.7e8 at N=16384; measured 2.8e-11 relative there)
    assert abs(rb - float(s["res_after"])) <= 1e-10 * float(s["res_after"])
    uf, rf = out[_lib.FP_FMA]
    assert float(np.max(np.abs(uf - ub))) <= 1e-12
    assert abs(rf - rb) <= 1e-9 * rb


@pytest.mark.slow
def test_two_timesteps_N16384(golden_summary):
    s = golden_summary["steps"].get("N16384_L9_2steps")
    if s is None:
        pytest.skip("large fixture not generated")
    N, maxlvl = 16384, 9
    u0, v1, v2 = init_problem(N)
    dt = 1.0 / N / 10
    with Multigrid(N, maxlvl, dt, NU) as mg:
        mg.upload(u0, v1, v2)
        del v1, v2
        cyc = [mg.step(1e-6) for _ in range(2)]
        u = mg.download(u0)
    assert cyc == [3, 3]
    assert hashlib.sha256(u.tobytes()).hexdigest() == s["sha256"]


@pytest.mark.parametrize("N,maxlvl,nsmooth,shape,tower", [
    (4096, 3, 2, 1, 0),     # config 2: 3-level V-cycle, 2 pre/post sweeps
    (512, 4, 3, 2, 0),      # W-cycle (multigrid.cpp:52)
    (512, 5, 3, 1, 1),      # correct tower
    (1024, 5, 3, 2, 1),     # correct tower, W-cycle (fused coarsest solve, pair passes)
    (256, 7, 1, 1, 0),      # coarsest n = 4
    (2048, 2, 3, 1, 0),     # large coarsest level (host-loop coarse solve)
])
def test_mg_outer_bitwise_vs_oracle(oracle_mod, N, maxlvl, nsmooth, shape, tower, tile_mode):
    O = oracle_mod
    O.set_threads(8)
    try:
        u0, v1, v2 = init_problem(N)
        dt = 1.0 / N / 10
        t = O.Tower(u0, v1, v2, N, maxlvl, tower)
        O.compute_rhs(t.ufine, N, v1, v2, dt, NU, 1.0 / N, rhs=t.rhsfine)
        cyc_ref, r0_ref, r_ref = t.mg_outer(dt, NU, 1e-6, shape, nsmooth)
        with Multigrid(N, maxlvl, dt, NU, nsmooth=nsmooth, shape=shape, tower_mode=tower) as mg:
            mg.upload(u0, v1, v2)
            mg.rhs()
            cyc, r0, r, _ = mg.mg_outer(1e-6)
            assert cyc == cyc_ref
            assert abs(r0 - r0_ref) <= 1e-11 * r0_ref
            # final norm comes from the residual stage fused into the last
            # post-smoothing pass
            assert abs(r - r_ref) <= 1e-11 * r_ref
            assert np.array_equal(mg.download(), t.ufine)
    finally:
        O.set_threads(1)


def test_maxlvl1_fine_level_is_coarsest():
    """N=32 default maxlvl = 1: mg_inner solves the fine grid by GS (K4: 2 cycles)."""
    g = load_golden("e2e_N32.npz")
    assert set(g["cycles"]) == {2}


def test_run_cycles_is_deterministic():
    N, maxlvl = 1024, 5
    u0, v1, v2 = init_problem(N)
    dt = 1.0 / N / 10
    outs = []
    for _ in range(2):
        with Multigrid(N, maxlvl, dt, NU) as mg:
            mg.upload(u0, v1, v2)
            mg.rhs()
            r = mg.run_cycles(3)
            outs.append((mg.download(), r))
    assert np.array_equal(outs[0][0], outs[1][0]) and outs[0][1] == outs[1][1]


@pytest.mark.parametrize("N", [64, 128])
def test_coarsest_solve_to_rounding_matches_direct_solve(N):
    """SURVEY 8f item 4 (the intent of exact_solve.cpp): the coarsest-level
    solve driven to rounding (coarse_tol -> 1e-13) equals a sparse direct
    solve of the same Crank-Nicolson operator (gs.cpp:126-130 coefficients,
    level velocities, Dirichlet 0) to 1e-12 relative."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla
    u0, v1, v2 = init_problem(N)
    dt, h = 1.0 / N / 10, 1.0 / N
    with Multigrid(N, 1, dt, NU, coarse_tol=1e-13, coarse_maxit=1000) as mg:
        mg.upload(u0, v1, v2)
        mg.rhs()
        rhs = mg.download_level(0, "rhs").reshape(N + 1, N + 1)
        mg.mg_inner()
        u = mg.download().reshape(N + 1, N + 1)
        iters = mg.coarse_iterations()
    V1, V2 = v1.reshape(N + 1, N + 1), v2.reshape(N + 1, N + 1)
    rr = 0.5 * dt / (h * h)
    a = lambda v: rr * (-v * h / 2.0 + NU)
    b = lambda v: rr * (v * h / 2.0 + NU)
    m = N - 1
    idx = lambda i, j: (i - 1) * m + (j - 1)
    rows, cols, vals = [], [], []
    for i in range(1, N):
        for j in range(1, N):
            k = idx(i, j)
            rows.append(k); cols.append(k); vals.append(1.0 - 4.0 * rr * NU)
            for (ii, jj, cf) in ((i - 1, j, a(V1[i, j])), (i, j - 1, a(V2[i, j])),
                                 (i + 1, j, b(V1[i, j])), (i, j + 1, b(V2[i, j]))):
                if 1 <= ii <= N - 1 and 1 <= jj <= N - 1:
                    rows.append(k); cols.append(idx(ii, jj)); vals.append(cf)
    A = sp.csr_matrix((vals, (rows, cols)), shape=(m * m, m * m))
    x = spla.spsolve(A.tocsc(), rhs[1:N, 1:N].ravel())
    err = np.max(np.abs(u[1:N, 1:N].ravel() - x)) / np.max(np.abs(x))
    assert err <= 1e-12, (err, iters)
    assert iters < 1000


def test_config2_bitwise_vs_nu2_reference(golden_summary):
    """BASELINE configs[1]: N=4096, 3-level V-cycle, 2 pre/post RB-GS sweeps
    (coarsest n=1024 solved by GS to 1e-5) against the reference built with
    NITER=2: one V-cycle and two Crank-Nicolson steps, sha256 + cycle counts."""
    N, L = 4096, 3
    dt = 1.0 / N / 10
    u0, v1, v2 = init_problem(N)
    sv = golden_summary["vcycle"]["N4096_L3_nu2"]
    with Multigrid(N, L, dt, NU, nsmooth=2) as mg:
        mg.upload(u0, v1, v2)
        mg.rhs()
        mg.mg_inner()
        assert hashlib.sha256(mg.download().tobytes()).hexdigest() == sv["sha256"]
        r = mg.residual_norm(0)
        assert abs(r - float(sv["res_after"])) <= 1e-11 * float(sv["res_after"])
    st = golden_summary["steps"]["N4096_L3_nu2_2steps"]
    with Multigrid(N, L, dt, NU, nsmooth=2) as mg:
        mg.upload(u0, v1, v2)
        cyc = [mg.step(1e-6) for _ in range(st["steps"])]
        assert cyc == st["cycles"]
        assert hashlib.sha256(mg.download().tobytes()).hexdigest() == st["sha256"]


@pytest.mark.parametrize("N,G,fuse", [(1024, 1, 1), (1024, 4, 1), (4096, 1, 1), (4096, 1, 0),
                                      (8192, 1, 1)],
                         ids=["N1024", "N1024_G4", "N4096", "N4096_nofuse", "N8192"])
def test_step_fused_rhs_norm_equals_rhs_then_mg_outer(N, G, fuse):
    """mgx_step computes compute_rhs and mg_outer's initial residual norm in
    one pass (k_res_march<3>), and on a row-march finest level (n >= 4096)
    the first cycle's pre-smoothing in the same pass too (k_wsmooth mode
    kModeRhsNorm, tuning key step_fuse); rhs() + mg_outer() runs them as
    separate passes.  Same cycle counts and bitwise the same u over three
    time steps, on one GPU and on row blocks."""
    L = 6
    dt, tol = 1.0 / N / 10, 1e-6
    u0, v1, v2 = init_problem(N)
    kw = dict(local_parts=G) if G > 1 else {}
    out = []
    old = _lib.get_tuning("step_fuse")
    _lib.set_tuning("step_fuse", fuse)
    try:
        for fused in (False, True):
            with Multigrid(N, L, dt, NU, **kw) as mg:
                mg.upload(u0, v1, v2)
                cyc = []
                for _ in range(3):
                    if fused:
                        cyc.append(mg.step(tol))
                    else:
                        mg.rhs()
                        cyc.append(mg.mg_outer(tol)[0])
                out.append((cyc, mg.download()))
    finally:
        _lib.set_tuning("step_fuse", old)
    assert out[0][0] == out[1][0]
    assert np.array_equal(out[0][1], out[1][1])


@pytest.mark.parametrize("N,maxlvl,nsmooth,tol,G,min_rows", [
    (4096, 5, 3, 1e-6, 1, 0), (4096, 4, 2, 1e-8, 1, 0), (8192, 6, 3, 1e-6, 1, 0),
    (4096, 5, 3, 1e-6, 4, 0),        # row blocks, levels 0-2 partitioned
    (4096, 4, 3, 1e-6, 2, 8192)],    # every level replicated (la = 0)
    ids=["N4096", "N4096nu2", "N8192", "N4096_G4", "N4096_G2_replicated"])
def test_post_predict_recompute_is_bitwise(N, maxlvl, nsmooth, tol, G, min_rows):
    """mg_outer skips storing u_post on cycles predicted not to converge and
    recomputes it (prolongation + post-smoothing of the cycle's input) when
    one converges anyway, and runs the cycle predicted to be the last as a
    post-smoothing pass without the next cycle's pre-smoothing: post_predict
    -1 (never store, always recompute), the defaults, post_only -1 (every
    cycle post-only) and 0 / 0 (always the cross pass, always store) give the
    same cycle counts and u, bitwise, and norms to 1e-11, over three time
    steps -- on one GPU and on virtual row blocks."""
    dt = 1.0 / N / 10
    u0, v1, v2 = init_problem(N)
    old = _lib.get_tuning("post_predict")
    old_po = _lib.get_tuning("post_only")
    old_rows = _lib.get_tuning("dist_min_rows")
    kw = dict(local_parts=G) if G > 1 else {}
    out = []
    try:
        if min_rows:
            _lib.set_tuning("dist_min_rows", min_rows)
        # (post_predict, post_only): always store / never post-only first, then
        # never store (recompute), the defaults, every cycle post-only (each
        # next cycle pre-smooths from u_post)
        for pp, po in ((0, 0), (-1, 0), (10, 10), (10, -1)):
            _lib.set_tuning("post_predict", pp)
            _lib.set_tuning("post_only", po)
            with Multigrid(N, maxlvl, dt, NU, nsmooth=nsmooth, **kw) as mg:
                if G > 1:
                    assert mg.dist_info()[2] == (0 if min_rows else 3)
                mg.upload(u0, v1, v2)
                res = []
                for _ in range(2):
                    mg.rhs()
                    res.append(mg.mg_outer(tol)[:3])
                res.append(mg.step(tol))
                out.append((res, mg.download()))
    finally:
        _lib.set_tuning("post_predict", old)
        _lib.set_tuning("post_only", old_po)
        _lib.set_tuning("dist_min_rows", old_rows)
    for res, u in out[1:]:
        assert [r[0] for r in res[:2]] == [r[0] for r in out[0][0][:2]]
        assert res[2] == out[0][0][2]
        np.testing.assert_allclose(np.array([r[1:] for r in res[:2]]),
                                   np.array([r[1:] for r in out[0][0][:2]]), rtol=1e-11)
        assert np.array_equal(u, out[0][1])


@pytest.mark.parametrize("post_only", [10, -1], ids=["default", "every_cycle"])
def test_step_cross_prepares_next_step_bitwise(post_only):
    """mgx_step's last cycle runs the cross pass in time-step mode: wave B
    forms the NEXT step's rhs from u_post, its initial norm, its first
    pre-smoothing and restriction, and the next mgx_step starts from that
    (step_cross = 1) -- against each step's own rhs + norm pass (0): the same
    cycle counts and u bitwise over four steps, the rhs of the last step
    bitwise; post_only = -1 runs step mode on every cycle, so every cycle but
    the last of a step mispredicts and falls back (pre-smoothing from u_post
    with the step's own rhs)."""
    N, L = 8192, 6
    dt, tol = 1.0 / N / 10, 1e-6
    u0, v1, v2 = init_problem(N)
    old = {k: _lib.get_tuning(k) for k in ("step_cross", "post_only")}
    out = []
    try:
        _lib.set_tuning("post_only", post_only)
        for sc in (0, 1):
            _lib.set_tuning("step_cross", sc)
            with Multigrid(N, L, dt, NU) as mg:
                mg.upload(u0, v1, v2)
                mg.profile(True, finest_only=True)
                cyc = [mg.step(tol) for _ in range(4)]
                rhs_passes = mg.profile_get(_lib.K_RHS, 0)[0]
                mg.profile(False)
                out.append((cyc, mg.download(), mg.download_level(0, "rhs"), rhs_passes))
    finally:
        for k, v in old.items():
            _lib.set_tuning(k, v)
    (c0, u0_, r0_, n0), (c1, u1_, r1_, n1) = out
    assert c0 == c1
    assert np.array_equal(u0_, u1_) and np.array_equal(r0_, r1_)
    assert n0 == 4 and n1 == 1   # one rhs + norm pass, the first step's


def test_step_cross_state_dropped_by_other_calls():
    """The next-step state a step leaves is used only by the next mgx_step:
    an upload, rhs + mg_outer or run_cycles in between drop it (each gives
    what it gives on a fresh context)."""
    N, L = 8192, 6
    dt, tol = 1.0 / N / 10, 1e-6
    u0, v1, v2 = init_problem(N)
    with Multigrid(N, L, dt, NU) as fresh:
        fresh.upload(u0, v1, v2)
        ref_step = [fresh.step(tol) for _ in range(2)]
        ref_u = fresh.download()
        fresh.upload(u0, v1, v2)
        fresh.rhs()
        ref_outer = fresh.mg_outer(tol)[0]
        ref_outer_u = fresh.download()
    with Multigrid(N, L, dt, NU) as mg:
        mg.upload(u0, v1, v2)
        mg.step(tol)                      # leaves the next step's state
        mg.upload(u0, v1, v2)             # ... which the upload drops
        assert [mg.step(tol) for _ in range(2)] == ref_step
        assert np.array_equal(mg.download(), ref_u)
        mg.upload(u0, v1, v2)
        mg.step(tol)
        mg.upload(u0, v1, v2)
        mg.rhs()
        assert mg.mg_outer(tol)[0] == ref_outer
        assert np.array_equal(mg.download(), ref_outer_u)
