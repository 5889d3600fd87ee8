"""GPU parity of the cross-cycle fused finest-level pass (k_xsmooth).

Inside mg_outer / run_cycles the post-smoothing of V-cycle k and the
pre-smoothing of cycle k+1 run as one HBM pass (tuning key "cross_cycle").
Bar: u after any number of cycles, the cycle counts and the per-cycle
norms are those of the unfused schedule -- u BITWISE, norms to 1e-11
(summation order of the partial sums); and every other entry point sees
the state it would without the fusion.
"""
import numpy as np
import pytest

from hpcclassmultigridproject_amd import Multigrid, _lib, init_problem

pytestmark = pytest.mark.gpu
NU = -4e-4
NORM_RTOL = 1e-11


@pytest.fixture
def cross():
    old = _lib.get_tuning("cross_cycle")
    yield lambda v: _lib.set_tuning("cross_cycle", v)
    _lib.set_tuning("cross_cycle", old)


def _cycles(N, L, n, cross_on, setter, **kw):
    setter(cross_on)
    u0, v1, v2 = init_problem(N)
    with Multigrid(N, L, 1.0 / N / 10, NU, **kw) as mg:
        mg.upload(u0, v1, v2)
        mg.rhs()
        mg.profile(True)
        norms = [mg.run_cycles(1) for _ in range(n)]
        xs = mg.profile_get(_lib.K_XSMOOTH)[0]
        mg.profile(False)
        return mg.download(), norms, xs


@pytest.mark.parametrize("N,L,kw", [(4096, 6, {}), (4096, 7, dict(nsmooth=2)),
                                    (8192, 5, {}), (4096, 3, {})],
                         ids=["N4096", "N4096nu2", "N8192", "N4096L3"])
def test_cross_cycle_equals_unfused(N, L, kw, cross):
    u_ref, n_ref, x_ref = _cycles(N, L, 4, 0, cross, **kw)
    u_x, n_x, x_x = _cycles(N, L, 4, 1, cross, **kw)
    assert x_ref == 0 and x_x == 4   # one cross pass per cycle
    assert np.array_equal(u_x, u_ref)
    np.testing.assert_allclose(n_x, n_ref, rtol=NORM_RTOL)


def test_cross_cycle_mg_outer_and_steps(cross):
    """mg_outer cycle counts, the returned u, and state across rhs/steps."""
    N, L = 4096, 6
    dt = 1.0 / N / 10
    u0, v1, v2 = init_problem(N)
    out = {}
    for on in (0, 1):
        cross(on)
        with Multigrid(N, L, dt, NU) as mg:
            mg.upload(u0, v1, v2)
            cyc = [mg.step(1e-6) for _ in range(3)]
            r0 = mg.residual_norm(0)
            mg.mg_inner()            # op-level V-cycle after fused cycles
            u = mg.download()
            cyc2, res0, res, _ = mg.mg_outer(1e-9)
            out[on] = (cyc, r0, u, cyc2, res0, res, mg.download())
    (c0, r00, u0_, c20, s00, s0, uf0), (c1, r01, u1_, c21, s01, s1, uf1) = out[0], out[1]
    assert c0 == c1 and c20 == c21
    assert np.array_equal(u0_, u1_) and np.array_equal(uf0, uf1)
    for a, b in ((r00, r01), (s00, s01), (s0, s1)):
        assert abs(a - b) <= NORM_RTOL * abs(a)


def test_run_cycles_batch_equals_single_calls(cross):
    """run_cycles(K) skips writing the intermediate cycles' solutions (only
    their norms are observed); the final state and norm must be identical."""
    cross(1)
    N, L = 4096, 6
    u0, v1, v2 = init_problem(N)
    out = []
    for batch in (False, True):
        with Multigrid(N, L, 1.0 / N / 10, NU) as mg:
            mg.upload(u0, v1, v2)
            mg.rhs()
            if batch:
                r = mg.run_cycles(4)
            else:
                for _ in range(4):
                    r = mg.run_cycles(1)
            r_after = mg.residual_norm(0)
            out.append((mg.download(), r, r_after))
    (ua, ra, raa), (ub, rb, rab) = out
    assert np.array_equal(ua, ub)
    assert ra == rb and raa == rab


def _cycles_plain(N, L, n, **kw):
    u0, v1, v2 = init_problem(N)
    with Multigrid(N, L, 1.0 / N / 10, NU, **kw) as mg:
        mg.upload(u0, v1, v2)
        mg.rhs()
        norms = [mg.run_cycles(1) for _ in range(n)]
        return mg.download(), norms


@pytest.mark.parametrize("xt", [0, 8193], ids=["edge_march", "edge_tiles"])
@pytest.mark.parametrize("N,L,G", [(4096, 6, 1), (8192, 5, 1), (4096, 6, 4), (4096, 6, 8)],
                         ids=["N4096", "N8192", "N4096_G4", "N4096_G8"])
def test_unguarded_interior_kernel_equals_guarded(N, L, G, xt, cross, knobs):
    """Tuning key "xfast": 1 = the cross pass runs as the unguarded interior
    kernel + the edges (boundary strips, top / bottom bands) as the guarded
    march ("xtile_max_rows" 0) or as LDS tiles (k_xtile, row blocks up to
    8193 rows); 0 = one guarded launch over the level.  u bitwise, norms to
    the summation-order tolerance; also on row blocks (virtual ranks, whose
    bands sit only at the first / last block; at G=8 the 512-row blocks are
    short enough to run entirely as tiles)."""
    cross(1)
    kw = dict(local_parts=G) if G > 1 else {}
    knobs(xfast=0)
    u0_, n0 = _cycles_plain(N, L, 3, **kw)
    knobs(xfast=1, xtile_max_rows=xt)
    u1_, n1 = _cycles_plain(N, L, 3, **kw)
    assert np.array_equal(u0_, u1_)
    np.testing.assert_allclose(n1, n0, rtol=NORM_RTOL)


@pytest.mark.parametrize("store_post", [False, True], ids=["pre_only", "post_too"])
def test_edge_tiles_store_post_vs_checker(store_post, cross, knobs, oracle_mod):
    """The edge tiles also write u_post when the cycle's solution is observed
    (single run_cycles calls; a batch writes only the last): two cycles,
    bitwise vs the checker's mg_inner."""
    cross(1)
    knobs(xfast=1, xtile_max_rows=8193)
    N, L = 4096, 5
    dt = 1.0 / N / 10
    u0, v1, v2 = init_problem(N)
    with Multigrid(N, L, dt, NU) as mg:
        mg.upload(u0, v1, v2)
        mg.rhs()
        if store_post:
            mg.run_cycles(1)
            mg.run_cycles(1)
        else:
            mg.run_cycles(2)
        u = mg.download()
    O = oracle_mod
    O.set_threads(8)
    t = O.Tower(u0, v1, v2, N, L)
    O.compute_rhs(t.ufine, N, v1, v2, dt, NU, 1.0 / N, rhs=t.rhsfine)
    for _ in range(2):
        t.mg_inner(dt, NU)
    assert np.array_equal(u, t.ufine)


@pytest.fixture
def knobs():
    """Set tuning keys for one test; restores the previous values."""
    saved = {}

    def set_(**kv):
        for k, v in kv.items():
            saved.setdefault(k, _lib.get_tuning(k))
            _lib.set_tuning(k, v)
    yield set_
    for k, v in saved.items():
        _lib.set_tuning(k, v)


@pytest.mark.parametrize("N,L,G", [(8192, 5, 1), (4096, 6, 4)], ids=["N8192", "N4096_G4"])
def test_work_order_does_not_change_results(N, L, G, cross, knobs):
    """march_order (band-major rows, XCD-contiguous workgroups), tile_xcd /
    tile32_min_n (tile order and 32-row tiles) only reorder the work: u
    bitwise, norms to the summation-order tolerance, on one GPU and on row
    blocks."""
    cross(1)
    kw = dict(local_parts=G) if G > 1 else {}
    knobs(march_order=0, tile_xcd=0, tile32_min_n=1 << 30)
    u_ref, n_ref = _cycles_plain(N, L, 3, **kw)
    for mo, tx, t32 in ((1, 0, 1 << 30), (2, 1, 0), (3, 1, 1024)):
        knobs(march_order=mo, tile_xcd=tx, tile32_min_n=t32)
        u, n = _cycles_plain(N, L, 3, **kw)
        assert np.array_equal(u, u_ref), (mo, tx, t32)
        np.testing.assert_allclose(n, n_ref, rtol=NORM_RTOL)


@pytest.mark.parametrize("N,L,shape", [(4096, 7, 1), (1024, 6, 1), (256, 4, 1), (1024, 5, 2)],
                         ids=["c64", "c32", "c32s", "c64w"])
def test_coarse_solve_in_lds_equals_l2_version(N, L, shape, knobs):
    """coarse_lds: the coarsest solve with u in LDS and its constants in
    registers gives bitwise the u, norms and coarse iteration counts of the L2
    version (W-cycles: both solves of a visit in one launch)."""
    out = []
    u0, v1, v2 = init_problem(N)
    for v in (0, 1):
        knobs(coarse_lds=v)
        with Multigrid(N, L, 1.0 / N / 10, NU, shape=shape) as mg:
            mg.upload(u0, v1, v2)
            cyc = [mg.step(1e-6) for _ in range(2)]
            out.append((mg.download(), cyc, mg.coarse_iterations(), mg.residual_norm(0)))
    (ua, ca, ia, ra), (ub, cb, ib, rb) = out
    assert np.array_equal(ua, ub) and ca == cb and ia == ib and ra == rb


@pytest.mark.parametrize("N,L,shape,fp,parts", [
    (2048, 6, 1, _lib.FP_BITWISE, 0), (2048, 6, 2, _lib.FP_FMA, 0), (4096, 7, 2, _lib.FP_BITWISE, 0),
    (256, 3, 1, _lib.FP_FMA, 0), (1024, 5, 2, _lib.FP_FMA, 2)],
    ids=["V2048", "W2048fma", "W4096", "V256fma", "W1024fma_parts2"])
def test_coarse_fuse_equals_separate_launch(N, L, shape, fp, parts, knobs):
    """coarse_fuse: the coarsest solve (n = 64, u in LDS) inside the tile pass
    that prolongs from it -- every workgroup solves it in its LDS, workgroup 0
    stores it -- is bitwise the separate k_coarse_solve_lds launch: the
    solution, the norms, the coarse iteration counts and the coarsest level's
    stored u; no coarse launch remains."""
    out = []
    u0, v1, v2 = init_problem(N)
    for v in (0, 1):
        knobs(coarse_fuse=v)
        with Multigrid(N, L, 1.0 / N / 10, NU, shape=shape, fp_mode=fp,
                       local_parts=parts) as mg:
            mg.upload(u0, v1, v2)
            mg.rhs()
            mg.profile(True)
            norms = [mg.run_cycles(1) for _ in range(3)]
            cl = mg.profile_get(_lib.K_COARSE)[0]
            mg.profile(False)
            cyc = mg.step(1e-6)
            coarsest = None if parts else mg.download_level(L - 1)
            out.append((mg.download(), norms, cyc, mg.coarse_iterations(), coarsest, cl))
    (ua, na, ca, ia, za, la), (ub, nb, cb, ib, zb, lb) = out
    assert np.array_equal(ua, ub)
    assert na == nb and ca == cb and ia == ib
    if za is not None:
        assert np.array_equal(za, zb)
    assert la > 0 and lb == 0


@pytest.mark.parametrize("shape", [1, 2], ids=["V", "W"])
def test_coarse_fuse_nsmooth0_vs_oracle(shape, knobs, oracle_mod):
    """nsmooth = 0 (no smoothing, multigrid.cpp:69-88 with NITER 0): the
    prolongation is op_prolong_add, not a tile pass, so the coarsest solve must
    not be deferred into it -- coarse_fuse 0 and 1 bitwise equal, and equal to
    the CPU checker's mg_inner (advisor finding: with the solve deferred, the
    prolongation used to read the unsolved, zero coarse u)."""
    N, L = 1024, 5   # coarsest n = 64
    dt = 1.0 / N / 10
    u0, v1, v2 = init_problem(N)
    out = []
    for v in (0, 1):
        knobs(coarse_fuse=v)
        with Multigrid(N, L, dt, NU, shape=shape, nsmooth=0) as mg:
            mg.upload(u0, v1, v2)
            mg.rhs()
            for _ in range(2):
                mg.mg_inner()
            out.append((mg.download(), mg.coarse_iterations()))
    assert np.array_equal(out[0][0], out[1][0]) and out[0][1] == out[1][1]
    O = oracle_mod
    O.set_threads(8)
    t = O.Tower(u0, v1, v2, N, L)
    O.compute_rhs(t.ufine, N, v1, v2, dt, NU, 1.0 / N, rhs=t.rhsfine)
    for _ in range(2):
        t.mg_inner(dt, NU, shape=shape, nsmooth=0)
    assert np.array_equal(out[1][0], t.ufine)
    assert not np.array_equal(out[1][0], u0)   # the correction was applied


def test_wcycle_profile_counts_only_real_launches(knobs):
    """A W-cycle's pair pass declines on march levels (nothing launched); the
    profile must not count it: level 0 (n = 2048, a row march) runs exactly
    `shape` post-smoothing passes per cycle."""
    knobs(wpair=1)
    N, L = 2048, 6
    u0, v1, v2 = init_problem(N)
    with Multigrid(N, L, 1.0 / N / 10, NU, shape=2) as mg:
        mg.upload(u0, v1, v2)
        mg.rhs()
        mg.profile(True)
        for _ in range(2):
            mg.mg_inner()
        n0 = mg.profile_get(_lib.K_PSMOOTH, 0)[0]
        mg.profile(False)
    assert n0 == 2 * 2, n0


@pytest.mark.parametrize("N,L,shape,gl", [(4096, 7, 1, 3), (4096, 7, 2, 3), (2048, 6, 2, 1),
                                          (1024, 5, 1, 2)],
                         ids=["V4096_L3", "W4096_L3", "W2048_L1", "V1024_L2"])
def test_graph_replay_equals_launches(N, L, shape, gl, knobs):
    """graph_level: the sub-cycle below a level captured once per entry
    state as a hipGraph and replayed -- u, norms, cycle counts and coarse
    iterations bitwise the launched schedule's, through run_cycles, mg_inner
    and time steps (W-cycles: the pair passes and the fused coarsest solve
    with its second rhs buffer inside the graph)."""
    out = []
    u0, v1, v2 = init_problem(N)
    for v in (0, gl):
        knobs(graph_level=v)
        c0 = _lib.get_tuning("graph_captures")
        r0 = _lib.get_tuning("graph_replays")
        with Multigrid(N, L, 1.0 / N / 10, NU, shape=shape, fp_mode=_lib.FP_FMA) as mg:
            mg.upload(u0, v1, v2)
            mg.rhs()
            norms = [mg.run_cycles(1) for _ in range(2)] + [mg.run_cycles(3)]
            mg.mg_inner()
            cyc = [mg.step(1e-6) for _ in range(2)]
            out.append((mg.download(), norms, cyc, mg.coarse_iterations(),
                        _lib.get_tuning("graph_captures") - c0,
                        _lib.get_tuning("graph_replays") - r0))
    (ua, na, ca, ia, cap_a, rep_a), (ub, nb, cb, ib, cap_b, rep_b) = out
    assert np.array_equal(ua, ub)
    assert na == nb and ca == cb and ia == ib
    assert cap_a == 0 and rep_a == 0
    assert cap_b >= 1 and rep_b >= 1, (cap_b, rep_b)   # the graph path really ran


def test_negative_diagonal_routes_to_general_division(cross, oracle_mod):
    """nu > 0 large enough that the finest level's diagonal 1-4*rr*nu is
    negative: the unguarded cross kernel's division form assumes d > 0, so the
    launcher must run the level through the guarded kernel (general form, zero
    signs included).  Two cycles bitwise vs the unfused schedule and the
    checker (N=4096: rr = 204.8, nu = 0.002 -> d = -0.6384 on level 0)."""
    N, L, nu = 4096, 3, 0.002
    dt = 1.0 / N / 10
    u0, v1, v2 = init_problem(N)
    out = []
    for on in (0, 1):
        cross(on)
        with Multigrid(N, L, dt, nu) as mg:
            mg.upload(u0, v1, v2)
            mg.rhs()
            mg.run_cycles(2)
            out.append(mg.download())
    assert np.array_equal(out[0], out[1])
    O = oracle_mod
    O.set_threads(8)
    t = O.Tower(u0, v1, v2, N, L)
    O.compute_rhs(t.ufine, N, v1, v2, dt, nu, 1.0 / N, rhs=t.rhsfine)
    for _ in range(2):
        t.mg_inner(dt, nu)
    assert np.array_equal(out[1], t.ufine)


@pytest.mark.parametrize("N,L,G", [(8192, 6, 8), (4096, 6, 4)], ids=["N8192_G8", "N4096_G4"])
def test_one_segment_per_workgroup_plan(N, L, G, cross, knobs):
    """march_seg: on row blocks whose last band would be short, the marches
    give each workgroup one full-height segment instead of equal unit shares;
    only the work split changes: u bitwise, norms to the summation-order
    tolerance."""
    cross(1)
    kw = dict(local_parts=G)
    knobs(march_seg=0)
    u0_, n0 = _cycles_plain(N, L, 3, **kw)
    knobs(march_seg=1)
    u1_, n1 = _cycles_plain(N, L, 3, **kw)
    assert np.array_equal(u0_, u1_)
    np.testing.assert_allclose(n1, n0, rtol=NORM_RTOL)


@pytest.mark.parametrize("N,L,kw", [(4096, 4, {}), (4096, 5, dict(nsmooth=2)),
                                    (8192, 4, dict(fp_mode=_lib.FP_FMA))],
                         ids=["N4096", "N4096nu2", "N8192fma"])
def test_wcycle_cross_passes_equal_unfused(N, L, kw, cross):
    """W-cycles (shape 2, multigrid.cpp:52): the two level-0 visits of a cycle
    are fused (visit 1's post- with visit 2's pre-smoothing) and the last one
    with the next cycle's pre-smoothing -- two cross passes per W-cycle, u
    bitwise the unfused schedule's, norms to 1e-11."""
    u_ref, n_ref, x_ref = _cycles(N, L, 4, 0, cross, shape=2, **kw)
    u_x, n_x, x_x = _cycles(N, L, 4, 1, cross, shape=2, **kw)
    assert x_ref == 0 and x_x == 2 * 4
    assert np.array_equal(u_x, u_ref)
    np.testing.assert_allclose(n_x, n_ref, rtol=NORM_RTOL)


@pytest.mark.parametrize("nsmooth", [1, 2, 3])
@pytest.mark.parametrize("fp", [_lib.FP_BITWISE, _lib.FP_FMA], ids=["bitwise", "fma"])
def test_wcycle_tile_pairs_equal_unfused_and_oracle(oracle_mod, knobs, nsmooth, fp):
    """W-cycles on the LDS-tile levels: a visit's post-smoothing and the next
    visit's pre-smoothing as ONE tile pass (tuning key wpair, 2 nsmooth sweeps
    between the prolongation and the restriction) -- bitwise the two passes,
    and (bitwise mode) the CPU checker's mg_inner, multigrid.cpp:17-92 with
    shape 2.  The coarsest level's two solves per visit run in one launch."""
    N, L = 2048, 6   # levels 1..4 tiles (n <= 1024), coarsest 64
    out = {}
    for w in (0, 1):
        knobs(wpair=w)
        u0, v1, v2 = init_problem(N)
        with Multigrid(N, L, 1.0 / N / 10, NU, shape=2, nsmooth=nsmooth, fp_mode=fp) as mg:
            mg.upload(u0, v1, v2)
            mg.rhs()
            mg.profile(True)
            for _ in range(2):
                mg.mg_inner()
            launches = mg.profile_get(_lib.K_PSMOOTH)[0] + mg.profile_get(_lib.K_GS)[0]
            coarse = mg.profile_get(_lib.K_COARSE)[0]
            mg.profile(False)
            out[w] = (mg.download(), launches, coarse, mg.coarse_iterations())
    assert np.array_equal(out[1][0], out[0][0])
    assert out[1][3] == out[0][3]                  # the same coarse iterations
    assert out[1][1] < out[0][1], (out[0][1], out[1][1])
    # one launch per coarsest visit, or none with the solve fused into the
    # level above's prolongation pass (coarse_fuse, the default)
    assert out[0][2] == out[1][2] == (0 if _lib.get_tuning("coarse_fuse") else 2 * 2 ** (L - 1))
    if fp == _lib.FP_BITWISE:
        O = oracle_mod
        O.set_threads(8)
        dt = 1.0 / N / 10
        u0, v1, v2 = init_problem(N)
        t = O.Tower(u0, v1, v2, N, L)
        O.compute_rhs(t.ufine, N, v1, v2, dt, NU, 1.0 / N, rhs=t.rhsfine)
        for _ in range(2):
            t.mg_inner(dt, NU, shape=2, nsmooth=nsmooth)
        assert np.array_equal(out[1][0], t.ufine)


def test_wcycle_cross_vs_oracle_and_partitioned(oracle_mod, cross):
    """The fused W-cycle at N=4096 against the CPU checker's mg_inner (bitwise)
    and on 4 virtual row blocks (bitwise the one-GPU context)."""
    O = oracle_mod
    O.set_threads(8)
    N, L, cyc = 4096, 4, 2
    dt = 1.0 / N / 10
    cross(1)
    u0, v1, v2 = init_problem(N)
    t = O.Tower(u0, v1, v2, N, L)
    O.compute_rhs(t.ufine, N, v1, v2, dt, NU, 1.0 / N, rhs=t.rhsfine)
    for _ in range(cyc):
        t.mg_inner(dt, NU, shape=2)
    old = _lib.get_tuning("dist_min_rows")
    try:
        _lib.set_tuning("dist_min_rows", 16)
        outs = []
        for parts in (0, 4):
            with Multigrid(N, L, dt, NU, shape=2, local_parts=parts) as mg:
                mg.upload(u0, v1, v2)
                mg.rhs()
                mg.profile(True, finest_only=True)
                for _ in range(cyc):
                    mg.run_cycles(1)
                # (one launch per part: each virtual rank runs its own pass)
                assert mg.profile_get(_lib.K_XSMOOTH, 0)[0] == 2 * cyc * max(1, parts)
                outs.append(mg.download())
    finally:
        _lib.set_tuning("dist_min_rows", old)
    assert np.array_equal(outs[0], t.ufine)
    assert np.array_equal(outs[1], outs[0])
