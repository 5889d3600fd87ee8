"""GPU parity of the row-partitioned multi-GPU solver (dist.hip).

On the one-GPU test box the partition runs as G virtual ranks in one process
(``local_parts=G``: same partition plan, fused passes on row blocks with ghost
rows, ghost exchanges / all-gather as device copies).  RCCL itself is covered
with a world-size-1 communicator (the collectives' code path, no peers); the
real N-GPU RCCL run is the driver's multi-GPU bench.

Bar: u after V-cycles / mg_outer / timesteps is BITWISE the single-GPU result
and the reference's golden fixtures; cycle counts identical; residual norms
(per-rank partial sums, added across ranks) within 1e-11 relative of the
single-GPU tree sum (summation order only).
"""
import hashlib

import numpy as np
import pytest
from conftest import load_golden

from hpcclassmultigridproject_amd import MGXError, Multigrid, _lib, dist, init_problem

pytestmark = pytest.mark.gpu
NU = -4e-4
NORM_RTOL = 1e-11


@pytest.fixture
def min_rows(request):
    old = _lib.get_tuning("dist_min_rows")
    _lib.set_tuning("dist_min_rows", request.param)
    yield request.param
    _lib.set_tuning("dist_min_rows", old)


def _run(N, L, dt, nu, cycles, parts=0, **kw):
    u0, v1, v2 = init_problem(N)
    with Multigrid(N, L, dt, nu, local_parts=parts, **kw) as mg:
        mg.upload(u0, v1, v2)
        mg.rhs()
        norms = [mg.run_cycles(1) for _ in range(cycles)]
        u = mg.download()
        r = mg.residual_norm(0)
        info = mg.dist_info()
    return u, norms, r, info


@pytest.mark.parametrize("min_rows", [16], indirect=True)
@pytest.mark.parametrize("G", [2, 4])
def test_vcycle_partitioned_bitwise_vs_reference_N256(G, min_rows):
    g = load_golden("vcycle_N256_L4.npz")
    N, maxlvl, nu, dt = g["params"]
    N, maxlvl = int(N), int(maxlvl)
    u0, v1, v2 = init_problem(N)
    with Multigrid(N, maxlvl, dt, nu, local_parts=G) as mg:
        assert mg.dist_info() == (G, -1, maxlvl - 1)   # every non-coarsest level split
        mg.upload(u0, v1, v2)
        mg.rhs()
        mg.mg_inner()
        assert np.array_equal(mg.download(), g["u"])


@pytest.mark.parametrize("min_rows", [16, 256], indirect=True)
@pytest.mark.parametrize("G", [2, 4, 8])
def test_vcycles_partitioned_equal_single_N1024(G, min_rows):
    N, L = 1024, 6
    dt = 1.0 / N / 10
    us, ns, rs, _ = _run(N, L, dt, NU, 3)
    up, npart, rp, info = _run(N, L, dt, NU, 3, parts=G)
    assert info[0] == G
    assert np.array_equal(up, us)
    np.testing.assert_allclose(npart, ns, rtol=NORM_RTOL)
    assert abs(rp - rs) <= NORM_RTOL * rs


@pytest.mark.parametrize("min_rows", [128, 512], indirect=True)
@pytest.mark.parametrize("G", [2, 8])
def test_selfcheck_partitions_equal_single_N4096(G, min_rows):
    """The partitions bench.py's RCCL self-check runs for its candidates
    (N=4096, L=7, dist_min_rows 128 / 512; at G=8 and 512 only level 0 is
    split, la = 1) on virtual ranks: u bitwise the one-GPU context's, fma."""
    N, L = 4096, 7
    dt = 1.0 / N / 10
    fp = dict(fp_mode=_lib.FP_FMA)
    us, ns, rs, _ = _run(N, L, dt, NU, 3, **fp)
    up, npart, rp, info = _run(N, L, dt, NU, 3, parts=G, **fp)
    assert info[0] == G and info[2] >= 1
    assert np.array_equal(up, us)
    np.testing.assert_allclose(npart, ns, rtol=NORM_RTOL)


@pytest.mark.parametrize("G", [2, 4, 8])
def test_vcycle_partitioned_summary_N4096(golden_summary, G):
    """Default plan (blocks >= 256 rows): reference sha256 after one V-cycle."""
    s = golden_summary["vcycle"]["N4096_L3"]
    N, L = s["N"], s["maxlvl"]
    u0, v1, v2 = init_problem(N)
    with Multigrid(N, L, 1.0 / N / 10, NU, local_parts=G) as mg:
        mg.upload(u0, v1, v2)
        mg.rhs()
        mg.mg_inner()
        u = mg.download()
        assert hashlib.sha256(u.tobytes()).hexdigest() == s["sha256"]
        r = mg.residual_norm(0)
        assert abs(r - float(s["res_after"])) <= NORM_RTOL * float(s["res_after"])


@pytest.mark.parametrize("min_rows", [16], indirect=True)
@pytest.mark.parametrize("kw", [dict(shape=2), dict(nsmooth=2), dict(nsmooth=4),
                                dict(fuse=1), dict(fuse=2, nsmooth=5),
                                dict(tower_mode=_lib.TOWER_CORRECT)],
                         ids=["wcycle", "nu2", "nu4", "fuse1", "fuse2nu5", "correct_tower"])
def test_mg_outer_partitioned_variants(kw, min_rows):
    N, L = 512, 5
    dt = 1.0 / N / 10
    u0, v1, v2 = init_problem(N)
    out = []
    for parts in (0, 4):
        with Multigrid(N, L, dt, NU, local_parts=parts, **kw) as mg:
            mg.upload(u0, v1, v2)
            mg.rhs()
            cyc, r0, r, capped = mg.mg_outer(1e-6)
            out.append((mg.download(), cyc, r0, r, capped, mg.coarse_iterations()))
    (us, cs, r0s, rs, caps, its), (up, cp, r0p, rp, capp, itp) = out
    assert (cp, capp) == (cs, caps)
    assert itp == its
    assert np.array_equal(up, us)
    assert abs(r0p - r0s) <= NORM_RTOL * r0s and abs(rp - rs) <= NORM_RTOL * rs


@pytest.fixture(params=[2048, 0], ids=["tile", "march"])
def tile_mode(request):
    old = _lib.get_tuning("tile_max_n")
    _lib.set_tuning("tile_max_n", request.param)
    yield request.param
    _lib.set_tuning("tile_max_n", old)


@pytest.mark.parametrize("min_rows", [16], indirect=True)
def test_partitioned_tile_and_march_paths(tile_mode, min_rows):
    """Row blocks on the LDS-tile kernel levels and on the row-march levels."""
    N, L = 2048, 7
    dt = 1.0 / N / 10
    us, ns, _, _ = _run(N, L, dt, NU, 2)
    up, npart, _, _ = _run(N, L, dt, NU, 2, parts=8)
    assert np.array_equal(up, us)
    np.testing.assert_allclose(npart, ns, rtol=NORM_RTOL)


@pytest.mark.parametrize("min_rows", [16], indirect=True)
@pytest.mark.parametrize("tag", ["N128", "N128_nu001"])
def test_timesteps_partitioned_bitwise_vs_reference(tag, min_rows):
    """100 Crank-Nicolson steps (rhs + mg_outer each) on 2 row blocks."""
    g = load_golden(f"e2e_{tag}.npz")
    N, maxlvl, nu, dt, T, tol = g["params"]
    N, maxlvl = int(N), int(maxlvl)
    u0, v1, v2 = init_problem(N)
    with Multigrid(N, maxlvl, dt, nu, local_parts=2) as mg:
        mg.upload(u0, v1, v2)
        cyc = [mg.step(tol) for _ in range(int(T / dt))]
        uT = mg.download()
    assert cyc == list(g["cycles"])
    assert np.array_equal(uT, g["uT"])


def test_rccl_world1_equals_single():
    """mgx_create_dist on a size-1 RCCL communicator: the collective code path."""
    N, L = 1024, 6
    dt = 1.0 / N / 10
    uid = dist.unique_id()
    assert len(uid) == _lib.UNIQUE_ID_BYTES and any(uid)
    us, ns, rs, _ = _run(N, L, dt, NU, 2)
    u0, v1, v2 = init_problem(N)
    with Multigrid(N, L, dt, NU, world=1, rank=0, unique_id=uid) as mg:
        assert mg.dist_info() == (1, 0, L - 1)
        mg.upload(u0, v1, v2)
        mg.rhs()
        norms = [mg.run_cycles(1) for _ in range(2)]
        u = mg.download()
    assert np.array_equal(u, us)
    np.testing.assert_allclose(norms, ns, rtol=NORM_RTOL)


@pytest.mark.parametrize("min_rows", [16], indirect=True)
def test_partitioned_refuses_per_level_ops_and_profiles(min_rows):
    N, L = 256, 4
    u0, v1, v2 = init_problem(N)
    with Multigrid(N, L, 1.0 / N / 10, NU, local_parts=2) as mg:
        mg.upload(u0, v1, v2)
        for op in (lambda: mg.gs(0), lambda: mg.restrict(0), lambda: mg.prolong_add(0),
                   lambda: mg.download_level(1), lambda: mg.residual_norm(1)):
            with pytest.raises(MGXError):
                op()
        mg.profile(True)
        mg.rhs()
        mg.run_cycles(2)
        halo = mg.profile_get(_lib.K_HALO)
        coarse = mg.profile_get(_lib.K_COARSE)
        smooth = mg.profile_get(_lib.K_GS, 0)
        mg.profile(False)
    assert halo[0] > 0 and coarse[0] == 2 * 2   # 2 cycles x 2 replicas
    assert smooth[0] > 0 and smooth[1] > 0


def test_partitioned_create_errors():
    with pytest.raises(MGXError):   # world must be a power of two
        Multigrid(256, 4, 1e-3, NU, local_parts=3)
    with pytest.raises(MGXError):   # the partitioned path is the fused smoother
        Multigrid(256, 4, 1e-3, NU, local_parts=2, smoother=1)
    with pytest.raises(MGXError):
        Multigrid(256, 4, 1e-3, NU, local_parts=2, nsmooth=0)


@pytest.mark.parametrize("G", [2, 4, 8])
def test_cross_cycle_partitioned_equals_single_N4096(G):
    """Finest level >= 4096: the cross-cycle pass runs on the row blocks
    (16 ghost rows), in single-cycle calls, batched run_cycles and mg_outer."""
    N, L = 4096, 6
    dt = 1.0 / N / 10
    u0, v1, v2 = init_problem(N)
    out = []
    for parts in (0, G):
        with Multigrid(N, L, dt, NU, local_parts=parts) as mg:
            mg.upload(u0, v1, v2)
            mg.rhs()
            mg.profile(True)
            n1 = [mg.run_cycles(1) for _ in range(2)]
            n3 = mg.run_cycles(3)
            xs = mg.profile_get(_lib.K_XSMOOTH)[0]
            mg.profile(False)
            u_a = mg.download()
            cyc, r0, r, _ = mg.mg_outer(1e-10)
            out.append((n1, n3, xs, u_a, cyc, r0, r, mg.download()))
    s, p = out
    assert s[2] == 5 and p[2] == 5 * G   # one cross pass per cycle (per part)
    assert np.array_equal(p[3], s[3]) and np.array_equal(p[7], s[7])
    assert p[4] == s[4]
    np.testing.assert_allclose(p[0] + [p[1], p[5], p[6]], s[0] + [s[1], s[5], s[6]],
                               rtol=NORM_RTOL)


@pytest.mark.parametrize("N,L,G,min_rows", [(4096, 6, 4, 256), (1024, 6, 8, 16)],
                         indirect=["min_rows"], ids=["N4096G4", "N1024G8"])
def test_row_block_upload_equals_full_upload(N, L, G, min_rows):
    """mgx_upload_rows: every part gets only its rows (init_problem_rows) and
    the correct velocity tower is built on the device from the row blocks;
    the solve is bitwise the single-GPU one with the correct tower."""
    from hpcclassmultigridproject_amd import init_problem_rows
    dt = 1.0 / N / 10
    u0, v1, v2 = init_problem(N)
    with Multigrid(N, L, dt, NU, tower_mode=_lib.TOWER_CORRECT) as mg:
        mg.upload(u0, v1, v2)
        mg.rhs()
        n_ref = [mg.run_cycles(1) for _ in range(2)] + [mg.run_cycles(2)]
        u_ref = mg.download()
    with Multigrid(N, L, dt, NU, tower_mode=_lib.TOWER_CORRECT, local_parts=G) as mg:
        blocks = []
        for part in range(G):
            lo, hi = mg.dist_rows(part)
            blocks.append(init_problem_rows(N, lo, hi + 1))
        mg.upload_rows(blocks)
        mg.rhs()
        n_got = [mg.run_cycles(1) for _ in range(2)] + [mg.run_cycles(2)]
        u_got = mg.download()
    assert np.array_equal(u_got, u_ref)
    np.testing.assert_allclose(n_got, n_ref, rtol=NORM_RTOL)


def test_row_block_upload_refuses_reference_tower():
    with Multigrid(1024, 5, 1e-4, NU, local_parts=2) as mg:
        lo, hi = mg.dist_rows(0)
        from hpcclassmultigridproject_amd import init_problem_rows
        blk = init_problem_rows(1024, lo, hi + 1)
        with pytest.raises(MGXError):
            mg.upload_rows([blk, blk])


# ---- config C4: N=16384 row-partitioned (virtual ranks on the one-GPU box;
# the same partition plan and exchange plan the RCCL ranks execute)
@pytest.mark.slow
@pytest.mark.parametrize("G", [2, 4, 8])
def test_C4_vcycle_partitioned_N16384(golden_summary, G):
    """Headline size on G row blocks (levels 0..la-1 partitioned, the rest
    replicated): one V-cycle bitwise = the reference's sha256."""
    s = golden_summary["vcycle"]["N16384_L9"]
    N, L = 16384, 9
    u0, v1, v2 = init_problem(N, nthreads=16)
    with Multigrid(N, L, 1.0 / N / 10, NU, local_parts=G) as mg:
        assert mg.dist_info()[0] == G and mg.dist_info()[2] >= 3
        mg.upload(u0, v1, v2)
        del v1, v2
        mg.rhs()
        mg.mg_inner()
        u = mg.download(u0)
    assert hashlib.sha256(u.tobytes()).hexdigest() == s["sha256"]


@pytest.mark.slow
@pytest.mark.parametrize("G", [2, 4, 8])
def test_C4_two_timesteps_partitioned_N16384(golden_summary, G):
    """Two Crank-Nicolson steps (rhs + mg_outer with the cross-cycle pass on
    row blocks): cycles [3, 3] and the reference's sha256."""
    s = golden_summary["steps"]["N16384_L9_2steps"]
    N, L = 16384, 9
    u0, v1, v2 = init_problem(N, nthreads=16)
    with Multigrid(N, L, 1.0 / N / 10, NU, local_parts=G) as mg:
        mg.upload(u0, v1, v2)
        del v1, v2
        mg.profile(True, finest_only=True)
        cyc = [mg.step(1e-6) for _ in range(2)]
        xs = mg.profile_get(_lib.K_XSMOOTH)[0]
        ps = mg.profile_get(_lib.K_PSMOOTH, 0)[0]
        mg.profile(False)
        u = mg.download(u0)
    assert cyc == [3, 3]
    # the cross-cycle pass ran on every block in the first two cycles of each
    # step, the third (predicted last: tuning key post_only) as a post-smoothing
    # pass of its own
    assert xs == 4 * G and ps == 2 * G
    assert hashlib.sha256(u.tobytes()).hexdigest() == s["sha256"]


@pytest.fixture
def overlap():
    old = _lib.get_tuning("dist_overlap")
    yield lambda v: _lib.set_tuning("dist_overlap", v)
    _lib.set_tuning("dist_overlap", old)


@pytest.fixture(params=[0, 1], ids=["inline", "side_stream"])
def local_side(request):
    old = _lib.get_tuning("dist_local_side")
    _lib.set_tuning("dist_local_side", request.param)
    yield request.param
    _lib.set_tuning("dist_local_side", old)


@pytest.mark.parametrize("G", [2, 4, 8])
def test_overlapped_exchange_bitwise(G, overlap, local_side):
    """dist_overlap = 1 (finest ghost rows exchanged on a second stream behind
    the coarse levels) and 2 (plus the level-1 exchange beside the interior of
    the cross pass, the two ghost bands after it) give the same u bitwise as
    the serialised schedule and as one GPU, norms to the summation-order
    tolerance (the split pass sums its partials in another order); with the
    virtual ranks' exchanges inline (dist_local_side 0) and on the second
    stream (1: the RCCL transport's fork / join on one GPU)."""
    N, L = 4096, 7
    dt = 1.0 / N / 10
    us, ns, rs, _ = _run(N, L, dt, NU, 4)
    out = {}
    for ov in (0, 1, 2):
        overlap(ov)
        out[ov] = _run(N, L, dt, NU, 4, parts=G)
    for ov in (0, 1, 2):
        up, npart, rp, info = out[ov]
        assert info[0] == G
        assert np.array_equal(up, us), ov
        np.testing.assert_allclose(npart, ns, rtol=NORM_RTOL)


@pytest.mark.slow
def test_C4_two_timesteps_overlapped_N16384(golden_summary, overlap):
    """Config C4 with the overlapped exchange: 8 row blocks, two timesteps,
    cycles [3, 3] and the reference's sha256."""
    s = golden_summary["steps"]["N16384_L9_2steps"]
    N, L = 16384, 9
    overlap(1)
    u0, v1, v2 = init_problem(N, nthreads=16)
    with Multigrid(N, L, 1.0 / N / 10, NU, local_parts=8) as mg:
        mg.upload(u0, v1, v2)
        del v1, v2
        cyc = [mg.step(1e-6) for _ in range(2)]
        u = mg.download(u0)
    assert cyc == [3, 3]
    assert hashlib.sha256(u.tobytes()).hexdigest() == s["sha256"]


def test_overlap2_without_xfast_is_bitwise(overlap):
    """Round-3 advisor finding: dist_overlap = 2 with the unguarded kernels
    off (xfast = 0) has no split pass to run; the cross pass must then take
    its plain form (not skip the finest level) -- bitwise the one-GPU result,
    and no error."""
    N, L, G = 4096, 7, 4
    dt = 1.0 / N / 10
    old = _lib.get_tuning("xfast")
    try:
        _lib.set_tuning("xfast", 0)
        us, ns, rs, _ = _run(N, L, dt, NU, 3)
        overlap(2)
        up, npart, rp, info = _run(N, L, dt, NU, 3, parts=G)
    finally:
        _lib.set_tuning("xfast", old)
    assert np.array_equal(up, us)
    np.testing.assert_allclose(npart, ns, rtol=NORM_RTOL)
