/* mgx.h -- C ABI of the MI355X-native geometric-multigrid V-cycle (libmgx.so).
 *
 * Drop-in boundary for the reference's hot path (soniareilly/HPCClassMultigridProject):
 *   - the op-level seam gs.h:3-17 (gauss_seidel, residual, compute_norm,
 *     prolongation, restriction, compute_rhs), here on DEVICE pointers in the
 *     reference layout (row-major (n+1)^2 doubles, element (i,j) at i*(n+1)+j);
 *   - the solver-level functions multigrid.cpp:17 (mg_inner), :97 (mg_outer)
 *     and :124 (timestepper), here on a context that keeps the level towers
 *     resident in HBM (mgx_ctx), plus mgx_timestepper with the exact reference
 *     signature on HOST arrays.
 *
 * Conventions:
 *   - every function returns 0 on success and a non-zero MGX_E* code on
 *     failure; mgx_last_error() returns the message of the last failure on the
 *     calling thread;
 *   - the caller owns every buffer passed in; ops never allocate;
 *   - raw-pointer ops run on the HIP null stream and are ordered with other
 *     null-stream work; mgx_compute_norm synchronises (it returns a host value,
 *     like gs.cpp:86).  Context functions run on the context's own stream;
 *   - all arithmetic is fp64 with the reference's term order and no FMA
 *     contraction, so op results are bitwise equal to the serial reference
 *     (a context may opt into contracted smoothing passes: MGX_FP_FMA).
 */
#ifndef MGX_H
#define MGX_H

#ifdef __cplusplus
extern "C" {
#endif

#define MGX_OK 0
#define MGX_E_ARG 1     /* invalid argument (sizes, level, null pointer) */
#define MGX_E_HIP 2     /* a HIP runtime call failed */
#define MGX_E_RCCL 3    /* an RCCL call failed */
#define MGX_E_NOCONV 4  /* mg_outer hit its cycle cap (reported, not fatal) */
#define MGX_E_INTERNAL 5 /* an internal consistency check failed (a bug) */

const char *mgx_last_error(void);
int mgx_version(void);

/* ---------------------------------------------------------------------------
 * Op-level seam: replaces gs.h (reference gs.h:3-17, implementations gs.cpp).
 * Device pointers, reference layout.  k = dt, h = grid spacing at this level.
 * ------------------------------------------------------------------------- */

/* gs.h:9 / gs.cpp:109-189: one red-black Gauss-Seidel sweep, in place. */
int mgx_gauss_seidel(double *u, const double *rhs, long n, const double *v1,
                     const double *v2, double k, double nu, double h);
/* gs.h:3 / gs.cpp:55-83: res = rhs - A u on the interior; res boundary untouched. */
int mgx_residual(double *res, const double *u, const double *rhs, long n,
                 const double *v1, const double *v2, double k, double nu, double h);
/* gs.h:5 / gs.cpp:86-107: *norm = sqrt(sum of interior res^2).  Does not modify res. */
int mgx_compute_norm(const double *res, long n, double *norm);
/* gs.h:16 / gs.cpp:228-266: bilinear prolongation, up (2n+1)^2 <- u (n+1)^2. */
int mgx_prolongation(double *up, const double *u, long n);
/* gs.h:17 / gs.cpp:268-292: injection, u (n/2+1)^2 <- up (n+1)^2 (incl. boundary). */
int mgx_restriction(double *u, const double *up, long n);
/* gs.h:13 / gs.cpp:24-53: Crank-Nicolson right-hand side B u on the interior. */
int mgx_compute_rhs(double *rhs, const double *u, long n, const double *v1,
                    const double *v2, double k, double nu, double h);

/* multigrid.cpp:206-233: the reference problem on the host with the C library
 * (glibc) exp/sin/cos, so inputs are bitwise those of the reference: Gaussian
 * u0 (x0=.2, y0=.4, sigma=100) with zero boundary, v1 = -pi sin(pi x) cos(pi y),
 * v2 = pi cos(pi x) sin(pi y); x = i/N, y = j/N.  Arrays of (N+1)^2 doubles.
 * nthreads <= 0: all hardware threads. */
int mgx_init_problem(double *u0, double *v1, double *v2, long N, int nthreads);
/* Rows [r0, r1) only, into arrays of (r1-r0)*(N+1) doubles: bitwise those rows
 * of mgx_init_problem (for row-block uploads, mgx_upload_rows). */
int mgx_init_problem_rows(double *u0, double *v1, double *v2, long N, long r0, long r1,
                          int nthreads);

/* ---------------------------------------------------------------------------
 * Solver level.
 * ------------------------------------------------------------------------- */

/* Tower construction (multigrid.cpp:148-160). */
#define MGX_TOWER_REFERENCE 0 /* bitwise reference semantics (index quirk, zero fill) */
#define MGX_TOWER_CORRECT 1   /* every level injected from the level above */

typedef struct mgx_options {
    int nsmooth;        /* RB-GS sweeps before and after the coarse correction
                           (NITER, multigrid.cpp:41; reference 3) */
    int shape;          /* 1 = V-cycle, 2 = W-cycle (multigrid.cpp:52) */
    int tower_mode;     /* MGX_TOWER_* (default REFERENCE) */
    int device;         /* HIP device ordinal for this context */
    double coarse_tol;  /* coarsest-level GS stop, absolute (multigrid.cpp:60: 1e-5) */
    int coarse_maxit;   /* coarsest-level GS cap (multigrid.cpp:60: 1000) */
    int max_cycle;      /* mg_outer cycle cap (multigrid.cpp:94: 50) */
    int smoother;       /* 0 = temporally blocked passes of up to `fuse` sweeps with
                           the prolongation fused into the post-smoothing pass
                           (default); 1 = two in-place colour passes per sweep;
                           2 = one-pass single sweeps (no temporal blocking) */
    int fuse;           /* smoother 0: max RB sweeps per HBM pass, 1..3 (default 3) */
    int fp_mode;        /* MGX_FP_BITWISE (default) or MGX_FP_FMA, below */
} mgx_options;

/* Arithmetic of the smoothing passes (smoother 0: the fused row marches,
 * LDS tiles and the coarsest solve; the gs.h mirror ops, smoothers 1/2 and
 * compute_rhs are always bitwise).
 * MGX_FP_BITWISE: the reference's expressions term by term, no contraction,
 *   the correctly rounded division -- u bitwise equal to the serial reference.
 * MGX_FP_FMA: the operator divided by its diagonal and contracted: each
 *   update u = f/d + m_N uN + m_W uW + m_E uE + m_S uS as four fused
 *   multiply-adds (m = -coefficient/d), residuals d*(update - u) -- within a
 *   few ulp per operation of the reference (max|duT| <= 1e-12,
 *   the same cycle counts), independent of the kernel or row partition that
 *   computes a point.  The reference's own GPU build contracts too (nvcc
 *   defaults to -fmad=true, gs.cu). */
#define MGX_FP_BITWISE 0
#define MGX_FP_FMA 1

/* Fills *opt with the reference defaults. */
void mgx_default_options(mgx_options *opt);

/* multigrid.cpp:124-186 with the reference signature: host arrays u0, v1, v2
 * of (n+1)^2 doubles in, uT out.  Runs (int)(T/dt) Crank-Nicolson steps, each
 * compute_rhs + mg_outer, entirely on the GPU. */
int mgx_timestepper(double *uT, const double *u0, const double *v1, const double *v2,
                    double nu, int maxlvl, long n, double dt, double T, double dx,
                    double tol, int shape);
/* Same with options; cycles_per_step (may be NULL) gets mg_outer's cycle count
 * for every step (length (int)(T/dt)). */
int mgx_timestepper_ex(double *uT, const double *u0, const double *v1, const double *v2,
                       double nu, int maxlvl, long n, double dt, double T, double dx,
                       double tol, const mgx_options *opt, int *cycles_per_step);

/* Context: the level towers u/rhs/v1/v2 (multigrid.cpp:131-162) resident in HBM.
 * n = finest N (power of two), maxlvl = number of levels, dt, nu as in
 * timestepper.  Multi-GPU: see mgx_create_dist. */
typedef struct mgx_ctx mgx_ctx;

int mgx_create(mgx_ctx **ctx, long n, int maxlvl, double dt, double nu,
               const mgx_options *opt);
int mgx_destroy(mgx_ctx *ctx);

/* Host <-> device in the reference layout ((n+1)^2 row-major).  upload sets
 * u = u0, v1, v2 on the finest level and builds the coarse velocity tower;
 * download copies the finest u. */
int mgx_upload(mgx_ctx *ctx, const double *u0, const double *v1, const double *v2);
int mgx_download(mgx_ctx *ctx, double *u);
/* Device-pointer variants (reference layout, device memory). */
int mgx_upload_device(mgx_ctx *ctx, const double *u0, const double *v1, const double *v2);
int mgx_download_device(mgx_ctx *ctx, double *u);

/* compute_rhs on the finest level (multigrid.cpp:167). */
int mgx_rhs(mgx_ctx *ctx);
/* `sweeps` RB-GS sweeps on level `level` (gauss_seidel, multigrid.cpp:69-72). */
int mgx_gs(mgx_ctx *ctx, int level, int sweeps);
/* residual + compute_norm on `level` (multigrid.cpp:104-105, 62-63). */
int mgx_residual_norm(mgx_ctx *ctx, int level, double *norm);
/* residual on `level` restricted into rhs[level+1], and u[level+1] = 0
 * (multigrid.cpp:73-77). */
int mgx_restrict(mgx_ctx *ctx, int level);
/* u[level] += prolongation(u[level+1]) (multigrid.cpp:81-83). */
int mgx_prolong_add(mgx_ctx *ctx, int level);
/* One V- (or W-) cycle from the finest level: mg_inner(lvl=0) (multigrid.cpp:17-92). */
int mgx_vcycle(mgx_ctx *ctx);
/* mg_outer (multigrid.cpp:97-120): cycles until ||r||/||r0|| <= tol or the cap.
 * Any output pointer may be NULL.  Returns MGX_E_NOCONV when the cap is hit. */
int mgx_mg_outer(mgx_ctx *ctx, double tol, int *cycles, double *res0, double *res);
/* One timestep: mgx_rhs + mgx_mg_outer (multigrid.cpp:165-172). */
int mgx_step(mgx_ctx *ctx, double tol, int *cycles);
/* Bench step x `cycles`: V-cycle + residual + norm, no tolerance stop.
 * *res (may be NULL) receives the last residual norm. */
int mgx_run_cycles(mgx_ctx *ctx, int cycles, double *res);

/* Introspection. */
int mgx_level_n(mgx_ctx *ctx, int level, long *n);
/* Copy level `level`'s field (0=u, 1=rhs, 2=v1, 3=v2) to host, reference layout. */
int mgx_download_level(mgx_ctx *ctx, int level, int field, double *out);
/* Number of coarsest-level GS iterations performed since creation. */
int mgx_coarse_iterations(mgx_ctx *ctx, long *iters);
/* The HIP stream (hipStream_t) the context launches on. */
int mgx_stream(mgx_ctx *ctx, void **stream);
/* Waits for all of the context's work; a partitioned context's side-stream
 * exchanges included, so no RCCL operation of it is in flight on return (the
 * caller's own collectives may follow). */
int mgx_synchronize(mgx_ctx *ctx);

/* Process-wide tuning knobs.  "tile_max_n": levels with n <= value run the
 * fused smoothing pass as 2-D LDS tiles instead of the row march (default 1024).
 * "cross_cycle": 1 (default) fuses, inside mg_outer / run_cycles / step, the
 * finest level's post-smoothing of each V-cycle with the pre-smoothing of
 * the next into one HBM pass (levels with n >= 4096, V- and W-cycles -- a
 * W-cycle also fuses its two level-0 visits --, nsmooth 2 or
 * 3; bitwise the same results); after such a cycle the coarse levels hold
 * the next cycle's restricted rhs, not the last correction.  0 = off.
 * "dist_min_rows": partitioned solvers replicate every level whose row blocks
 * would be shorter than this (default 256, even, >= 16); read at creation.
 * "dist_overlap": partitioned contexts, 1 = every partitioned level's u
 * ghost rows are exchanged on a second stream as soon as the pass that wrote
 * them ends, hidden behind the coarser levels (the level's next pass waits for
 * it), and the cross pass's restricted level-1 rhs behind the norm's host
 * round trip; 2 = that, and the cross pass's remaining exchange (level-1 u) on
 * the second stream beside the pass's interior march, the two 16-row bands next
 * to the ghosts after it; 0 = every exchange on the compute stream; -1
 * (default) = 1 on an RCCL communicator, 0 on virtual ranks (one GPU, where
 * the side stream's copies compete with the passes).  Bitwise the same results.
 * Whatever the mode, a rank has ONE communicator and at most one RCCL
 * operation in flight: each is chained after the previous one by an event.
 * "dist_comm_chain": test hook, 1 (default) = that chain; 0 drops it so the
 * fake-RCCL test can show its happens-before check catching the overlap.
 * Never 0 with real peers.
 * "dist_local_side": virtual ranks only: 0 (default) runs the dist_overlap
 * exchanges at their early points on the compute stream (one device: no
 * second link to overlap with), 1 on the second stream as over RCCL.  Bitwise
 * the same results.
 * "xfast": 1 (default) runs the cross-cycle pass as an unguarded kernel over
 * the interior strips and rows plus a guarded kernel over the boundary strips
 * and bands; 0 = one guarded launch (bitwise the same results).
 * "march_tile_rows": a row block whose wave march would give each resident
 * workgroup fewer than this many rows runs as LDS tiles (default 16, >= 0).
 * "xtile_max_rows": on row blocks of at most this many rows (a rank of a
 * partitioned solver, a small level) the cross-cycle pass runs the boundary
 * strips and bands as LDS tiles instead of the guarded row march (latency
 * bound: ~0.15 ms whatever the block height); default 4097, 0 = never.
 * "march_order": work order of the row marches, bit 0 = band-major (the
 * workgroups of neighbouring strip groups march the same rows at the same
 * time, so their shared halo columns are fetched once; launches with >= 192
 * rows per workgroup), bit 1 = XCD-contiguous workgroup order; default 3.
 * "tile_xcd": 1 (default) deals the LDS tiles
 * XCD-contiguous.  "tile32_min_n": K=3 tile passes on levels n >= value use
 * 32-row tiles (default 2048).  "march_min_rows": fewest rows per workgroup
 * of a wave-march launch (default 32, >= 8).
 * "march_seg": 1 (default) gives each workgroup of a row march one
 * full-height segment when equal shares would leave a short last band whose
 * workgroups march pieces of several strips (row blocks of a partitioned
 * level); 0 = equal shares only.
 * "step_fuse": 1 (default) runs a time step's compute_rhs, mg_outer's initial
 * residual norm and the first cycle's finest pre-smoothing as one pass
 * (single GPU, cross-cycle schedule, row-march finest level); 0 = the rhs and
 * norm pass, then the pre-smoothing (bitwise the same results).
 * "post_predict": mg_outer / step let the cross-cycle pass store a cycle's
 * post-smoothed u (the value returned if that cycle converges) only when the
 * cycle's residual, extrapolated with the last cycle's reduction factor, is
 * within post_predict x tol; a cycle that converges without it is recomputed
 * by one post-smoothing pass (default 10; 0 = always store,
 * -1 = never store: bitwise the same results).
 * "post_only": a cycle of mg_outer / step whose extrapolated norm is within
 * tol / post_only (or the last cycle allowed) runs its finest post-smoothing
 * as a pass of its own instead of the cross-cycle pass (no pre-smoothing of a
 * next cycle that would not run); if it does not converge after all, the next
 * cycle pre-smooths from its result (default 10; 0 = never; -1 = every cycle).
 * "step_cross": 1 (default) lets mgx_step's last cycle (single GPU, whole
 * levels n >= 8192) run the cross-cycle pass in time-step mode: it also
 * forms the next step's rhs, initial norm and first pre-smoothing, which the
 * next mgx_step starts from (any other call in between drops them); 0 = each
 * step starts with its own rhs + norm pass.
 * "coarse_fuse": 1 (default) runs the coarsest solve (n <= 64, with
 * coarse_lds) inside the prolongation tile pass of the level above: every
 * workgroup of that pass solves the coarsest level in its LDS and prolongs
 * from the copy, one stores it -- no coarse launch, bitwise the same results,
 * norms and iteration counts; 0 = its own launch.  Single-GPU contexts and
 * the replicated levels of a partitioned one, when the level above runs as
 * LDS tiles and the coarsest is level 2 or deeper.
 * "coarse_lds": 1 (default) solves coarsest levels n <= 64 with u in LDS
 * and each thread's rhs / v1 / v2 in registers, 0 = through L2 (bitwise the
 * same).  A W-cycle's `shape` consecutive solves of the coarsest level run in
 * one launch either way.
 * "wpair": 1 (default) runs a W-cycle's post-smoothing of one visit and the
 * pre-smoothing of the next visit of an LDS-tile level (nothing runs between
 * them, multigrid.cpp:52) as one tile pass of 2 nsmooth sweeps; 0 = two
 * passes (bitwise the same).
 * None of them changes a bit of u or a cycle count; residual norms taken by
 * a different kernel (cross_cycle, post_only, step_fuse) agree to 1e-11
 * relative (other reduction trees; a cycle count could differ only on a norm
 * that far from tol). */
int mgx_set_tuning(const char *key, long value);
/* "sep_velocity": 1 (default) = a velocity field that is an exact rank-1
 * outer product in floating point, v[i][j] == a[i]*b[j] bitwise (the
 * reference's rotating flow, multigrid.cpp:221-222, is one), is detected at
 * upload and the finest level's cross pass reads its factors instead of the
 * 2-D v1 / v2 (two of its five input streams); 0 = always the 2-D arrays.
 * Bitwise the same results either way.
 * "zero_rows": 1 (default) = at upload, the rows from which every row of a
 * coarse level's v1 and v2 is zero (3/4 of each coarse level of the
 * reference tower) are found, and the row marches read them from
 * one L2-resident zero row instead of HBM; 0 = every row from HBM (bitwise
 * the same results).
 * "vgen": 1 (default) = levels 1-2 of the reference tower, whose v1 / v2 are
 * re-reads of the finest rank-1 field, and every level below the
 * coarsest of the correct tower (strided injections of it: v_l(i, j) =
 * fl(a[2^l i] * b[2^l j])), generate them in the V-cycle's 3-sweep smoothing
 * passes from the finest level's factors instead of reading them from HBM --
 * only when every entry of the level equals the generator's bits (checked at
 * upload, per level; on row blocks per block, ghost rows included); 0 = reads
 * them.  Bitwise the same. */
/* Host only: exact rank-1 factors of v (rows x (n+1), row-major):
 * returns 1 and fills a[rows], b[n+1] with fl(a[i]*b[j]) == v[i][j] (same
 * bits) and every nonzero |v|, |b| still normal after scaling by smin, else 0. */
int mgx_factor_velocity(const double *v, long rows, long n, double smin, double *a, double *b);
/* *factored: a bit mask (since round 4; before, 0 or 1 -- bit 0 keeps that
 * meaning): bit 0 = the context keeps velocity factors for its finest level;
 * bit l (l >= 1) = level l generates its velocity from them ("vgen": levels
 * 1-2 of the reference tower, any level below the coarsest of the correct
 * tower). */
int mgx_velocity_factored(mgx_ctx *ctx, int *factored);
int mgx_get_tuning(const char *key, long *value);
/* Build provenance, fixed when the library was compiled: the sha256 (hex) of
 * the kernel sources (csrc stencil.h, kernels.h, kernels.hip, wsmooth.hip,
 * xsmooth.hip, concatenated in that order -- the key the committed PMC
 * profiles are stamped with) and of every product source (those + ctx.h,
 * plan.h, sepvel.h, mgx.hip, dist.hip, include/mgx.h). */
const char *mgx_build_id(void);
const char *mgx_build_sources_id(void);

/* Per-kernel timing with HIP events on the context stream. */
#define MGX_K_GS 0             /* RB-GS sweep (one full red+black sweep) */
#define MGX_K_RESTRICT 1       /* residual restricted to the coarse rhs */
#define MGX_K_PROLONG 2        /* prolongation + add */
#define MGX_K_RESNORM 3        /* residual + norm partials */
#define MGX_K_COARSE 4         /* coarsest-level solve */
#define MGX_K_RHS 5            /* compute_rhs */
#define MGX_K_HALO 6           /* halo exchange (multi-GPU) */
#define MGX_K_PSMOOTH 7        /* prolongation + add fused into a smoothing pass */
#define MGX_K_XSMOOTH 8        /* finest level: post-smoothing of cycle k + pre-smoothing of k+1 */
#define MGX_K_COUNT 9
/* on: 0 off, 1 every launch, 2 finest-level launches only (two events per
 * recorded launch; mode 2 keeps the overhead off the small levels). */
int mgx_profile_enable(mgx_ctx *ctx, int on);
int mgx_profile_reset(mgx_ctx *ctx);
/* For kernel kind `kind` on level `level` (-1 = all levels): launches, summed
 * device milliseconds, summed algorithmic bytes (SURVEY 8d byte model). */
int mgx_profile_get(mgx_ctx *ctx, int kind, int level, long *launches, double *ms,
                    double *bytes);
/* The same plus the compulsory bytes of those launches: every array a launch
 * reads or writes counted once (the traffic floor of a fused pass, and the
 * roofline denominator bench.py reports). */
int mgx_profile_get_ex(mgx_ctx *ctx, int kind, int level, long *launches, double *ms,
                       double *bytes, double *cbytes);

/* ---- Row-partitioned multi-GPU solver ---------------------------
 * The finest levels are split into contiguous row blocks, one per rank, with
 * ghost rows refreshed once per fused smoothing pass; levels whose blocks
 * would be shorter than 256 rows are replicated on every rank (the restricted
 * rhs is all-gathered).  u after any number of V-cycles is bitwise the
 * single-GPU (and reference) result; the residual norm is an all-reduced sum.
 * A partitioned context takes every whole-solver call (upload/download of the
 * full grid, rhs, vcycle, mg_outer, step, run_cycles, residual_norm at level
 * 0); the per-level calls (gs, restrict, prolong_add, download_level) return
 * MGX_E_ARG.  Needs smoother 0, nsmooth >= 1, world a power of two. */
/* Measured streaming bandwidth (GB/s, read + write bytes) of a 16-B-per-lane
 * grid-stride kernel with `nin` input streams (1: copy; 4: the smoother's
 * shape, 4 in + 1 out) of `bytes_per_stream` each, `reps` launches timed with
 * HIP events: the practical HBM ceiling reported beside the 8 TB/s spec. */
int mgx_stream_bandwidth(long bytes_per_stream, int nin, int reps, double *GBs);

#define MGX_UNIQUE_ID_BYTES 128
/* RCCL unique id (128 bytes) made on one rank and shared with the others. */
int mgx_dist_unique_id(void *id128);
/* One rank of `world` (one process per GPU; select the GPU with opt->device).
 * Collective: every rank must call it with the same id, n, maxlvl, options. */
int mgx_create_dist(mgx_ctx **out, long n, int maxlvl, double dt, double nu,
                    const mgx_options *opt, int rank, int world, const void *id128);
/* `world` virtual ranks in this process on one GPU, ghost exchanges as
 * device copies (tests the partition on a single GPU). */
int mgx_create_local_dist(mgx_ctx **out, long n, int maxlvl, double dt, double nu,
                          const mgx_options *opt, int world);
/* Partition plan (host only): owned rows [*ra, *rb) of `level` on `rank`, and
 * the first replicated level (levels >= it are whole on every rank). */
int mgx_partition(long n, int maxlvl, int world, int rank, int level, int *ra, int *rb,
                  int *replicated_level);
/* Host-only: the ghost-row exchange plan of `rank` on `level` (both transports
 * execute it).  *count entries of 5 ints: peer, send_row, send_rows, recv_row,
 * recv_rows (global rows of the level: send rows [send_row, +send_rows) to
 * peer, receive rows [recv_row, +recv_rows) from it); 0 entries on replicated
 * levels or world 1.  cap = room in xfers (entries). */
int mgx_exchange_plan(long n, int maxlvl, int world, int rank, int level, int *count,
                      int *xfers, int cap);
/* Host-only: the all-gather into the first replicated level *level: `rank`
 * contributes rows [*row0, *row0 + *rows) of its restricted rhs (in place,
 * rank-major, equal counts). */
int mgx_gather_plan(long n, int maxlvl, int world, int rank, int *level, int *row0,
                    int *rows);
/* Allocated rows [*lo, *hi] (owned + ghosts) of the finest level of local part
 * `part` (0 on an RCCL rank; 0..world-1 for mgx_create_local_dist). */
int mgx_dist_rows(mgx_ctx *ctx, int part, int *lo, int *hi);
/* Row-block upload, so that no rank ever holds the whole grid (SURVEY 8e C5:
 * N=65536 on 8 GPUs): u0[i], v1[i], v2[i] hold rows [lo, hi] (mgx_dist_rows)
 * of local part i, (hi-lo+1)*(N+1) doubles each.  The velocity tower is built
 * on the device from the row blocks, which needs MGX_TOWER_CORRECT (the
 * reference tower reads the whole grid).  Collective. */
int mgx_upload_rows(mgx_ctx *ctx, const double *const *u0, const double *const *v1,
                    const double *const *v2);
/* Owned finest-level rows [*ra, *rb) of local part `part` (the last rank also
 * owns the boundary row N; a single-GPU context: part 0 = [0, N+1)). */
int mgx_owned_rows(mgx_ctx *ctx, int part, int *ra, int *rb);
/* Row-block download, the counterpart of mgx_upload_rows: the owned rows of
 * local part `part` into rows[(rb-ra)*(N+1)], reference layout.  No
 * communication and no whole-grid buffer on any rank (C5: N=65536). */
int mgx_download_rows(mgx_ctx *ctx, int part, double *rows);
/* The reference's uT text output (multigrid.cpp:269-284, "%d\t%d\t%f\n", i
 * outer, j inner) for rows [r0, r1) held in rows[(r1-r0)*(N+1)]; append != 0
 * appends.  Rank-ordered appends of each rank's owned rows give the file the
 * whole-grid writer gives, byte for byte.  nthreads <= 0: all host threads. */
int mgx_write_uT(const char *path, const double *rows, long N, long r0, long r1, int append,
                 int nthreads);
/* world size, rank (-1 for a local multi-part context; 0/1 for single GPU),
 * first replicated level (maxlvl for a single-GPU context). */
int mgx_dist_info(mgx_ctx *ctx, int *world, int *rank, int *replicated_level);

#ifdef __cplusplus
}
#endif
#endif /* MGX_H */
