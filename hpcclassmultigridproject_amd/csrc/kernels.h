// kernels.h -- internal launch interface of the CDNA4 stencil kernels.
//
// Two layouts:
//   * reference layout: row-major, row pitch n+1 (gs.cpp:44), used by the
//     raw-pointer gs.h mirror ops (scalar, one point per lane);
//   * tower layout: row pitch P = round_up(n+1, 16) doubles (rows 128-B
//     aligned, pair (2c, 2c+1) 16-B aligned) used by the context path, one
//     column pair per lane, 16-B loads/stores.
#pragma once
#include <hip/hip_runtime.h>

namespace mgx {

// Per-level Crank-Nicolson operator constants, computed on the host with the
// reference's own expressions: rr = 0.5*k/(h*h) (gs.cpp:9-11),
// dgs = 1.0-4.0*rr*nu (gs.cpp:130, :75), drhs = 1.0+4.0*rr*nu (gs.cpp:44).
struct Coef {
    double rr, nu, h, dgs, drhs, rdgs;   // rdgs = RN(1/dgs)
    unsigned dsign;                       // sign bit of dgs (high-word position)
    // fp_mode fma (MGX_FP_FMA): the operator divided by its diagonal, see
    // stencil.h "fp_mode fma".  g = rr/d, gn = g*nu, c2 = -2 gn.
    double g, gn, c2;
    int fm;   // 1: the smoothing passes run the contracted (fma) forms
};
// fm: the context's fp_mode (0 bitwise, 1 fma)
Coef make_coef(double k, double nu, double h, int fm = 0);

// row pitch of the tower layout: n+1 rounded up to 16 doubles (128 B)
long tower_pitch(long n);

// ---------------------------------------------------------------- reference layout
void launch_raw_gs_colour(double *u, const double *rhs, const double *v1, const double *v2,
                          long n, Coef c, int colour, hipStream_t s);
void launch_raw_residual(double *res, const double *u, const double *rhs, const double *v1,
                         const double *v2, long n, Coef c, hipStream_t s);
void launch_raw_rhs(double *rhs, const double *u, const double *v1, const double *v2, long n,
                    Coef c, hipStream_t s);
void launch_raw_prolongation(double *up, const double *u, long n, hipStream_t s);
// injection: dst[I*(m)+J] = src[2I*src_pitch + 2J], 0<=I,J<m; pitches in doubles
void launch_injection(double *dst, long dst_pitch, const double *src, long src_pitch, long m,
                      hipStream_t s);
// rows x cols block: dst[I*dst_pitch + J] = src[2I*src_pitch + 2J]
void launch_injection_rows(double *dst, long dst_pitch, const double *src, long src_pitch,
                           long rows, long cols, hipStream_t s);
// flags[i] = 1 if row i (columns 0..n) of the pitched field holds a nonzero value
void launch_row_nonzero(const double *v, long pitch, long n, int *flags, hipStream_t s);

// Sum of squares of the interior of an (n+1)^2 field with row pitch `pitch`,
// deterministic two-stage reduction; result written to *out (device) as sqrt.
// `partials` must hold norm_partials_size() doubles.
int norm_partials_size();
// bandwidth probe: nin (1 or 4) double2 input streams -> one output stream
void launch_stream(const double *a, const double *b, const double *c, const double *d,
                   double *o, long n2, int nin, int grid, hipStream_t s);
void launch_norm(const double *res, long n, long pitch, double *partials, double *out,
                 hipStream_t s);

// ---------------------------------------------------------------- tower layout
// One full red-black sweep, out of place: uout = GS(uin).  Every point of
// uout (boundary included) is written.  zero_in: uin is taken as all zeros.
void launch_gs_sweep(const double *uin, double *uout, const double *rhs, const double *v1,
                     const double *v2, long n, long pitch, Coef c, bool zero_in,
                     hipStream_t s);
// `sweeps` (1..3) red-black sweeps in one pass, out of place: uout = GS^k(u_in)
// where u_in = 0 (mode bit 1), uin, or uin + P(uc) (mode bit 2: prolongation
// of the coarse level uc (coarse n = n/2, pitch pitchc) added on load).
// Mode bit 4: the residual of uout at the even-even points is written to the
// coarse rhs rhsc (pitchc); mode bit 8: the residual norm of uout is written
// to *norm_out (partials: norm_partials_size() doubles).  Returns the number
// of workgroups launched, -1 for an unsupported (sweeps, mode).
constexpr int kSmoothMaxSweeps = 3;
enum : int { kModeZero = 1, kModeProlong = 2, kModeRestrict = 4, kModeNorm = 8 };
// Mode bit 16 (with kModeRestrict, row march only, sweeps 2-3): the rhs is
// computed from uin on the fly (compute_rhs, gs.cpp:44) and stored to rhs_out,
// and the residual norm of uin against it goes to *norm_out -- a time step's
// compute_rhs, mg_outer's initial norm and the first pre-smoothing in one pass.
constexpr int kModeRhsNorm = 16;
// Velocity generator of level l (stencil.h vg_col): its v1 / v2 entries from
// the finest level's exact factors -- level 1 or 2 of the reference tower
// (strided 0: the injection quirk's re-read), or any level >= 1 of the correct
// tower (strided 1: entry (i, j) = finest (2^l i, 2^l j))
struct VGen {
    const double2 *a = nullptr;   // (sa1[I], sa2[I]), I = 0..N; (+0, +0) at N+1
    const double *b1 = nullptr, *b2 = nullptr;   // finest sb1, sb2 (0..N used)
    int l = 1;
    int strided = 0;
};
// clear *ok (device int) unless every entry (i in [r0, r1], j <= n) of level
// g.l's fields v1, v2 (pitch; v + i*pitch = global row i) equals the
// generator's bits; r1 < 0: every row 0..n
void launch_vgen_check(const double *v1, const double *v2, long n, long pitch, VGen g, int *ok,
                       hipStream_t s, int r0 = 0, int r1 = -1);
// Row-block correct tower: a[i << l] = (v1(i, js1), v2(i, js2)) for rows
// i in [r0, r1] of level l (the finest row factors are columns js << l of the
// finest field, where the column factor is exactly 1: sepvel.h) -- the factors
// of rows another rank factored, read from this rank's exchanged ghost rows
void launch_vgen_fill_rows(double2 *a, const double *v1, const double *v2, long pitch, int l,
                           int js1, int js2, int r0, int r1, hipStream_t s);
// the coarsest solve with u in LDS (stencil.h coarse_lds_body): levels n <= 64
constexpr int kCoarseLdsMaxN = 64;
constexpr int kCoarseLdsNP = kCoarseLdsMaxN + 1;

// The coarsest level's solve fused into the tile pass above it (k_smooth_tile
// with prolongation): every workgroup solves the coarsest level in LDS
// (stencil.h coarse_lds_body, n <= kCoarseLdsMaxN) and prolongs from that
// copy; the workgroup of blockIdx 0 also stores u and the iteration counts.
// on = 0: the pass reads the coarse u from HBM (uc).
struct CoarseFuse {
    double *u = nullptr;
    const double *rhs = nullptr, *v1 = nullptr, *v2 = nullptr;
    long n = 0, pitch = 0;
    Coef c{};
    double tol = 0.0;
    int maxit = 0, zero_first = 0, reps = 0;
    double *stats = nullptr;
    int on = 0;
};

struct SmoothArgs {
    const double *uin;
    double *uout;
    const double *rhs, *v1, *v2;
    long n, pitch;
    Coef c;
    const double *uc;   // coarse u (PROLONG)
    double *rhsc;       // coarse rhs (RESTRICT)
    long pitchc;        // pitch of the coarse level
    double *partials;   // NORM
    double *norm_out;   // NORM: sqrt of the sum (norm_sqrt) or the plain sum
    double *rhs_out = nullptr;   // kModeRhsNorm: the computed rhs
    // rows >= vz of v1 AND v2 are all zeros (the reference tower's coarse
    // levels, SURVEY K2: 3/4 of every coarse level): the row march reads them
    // from zrow (one zero row of >= pitch doubles, L2-resident) instead of HBM
    const double *zrow = nullptr;
    int vz = 0x7fffffff;
    // vg.a set (level 1 or 2 of the reference tower, checked at upload): the
    // 3-sweep pre / post passes generate v1, v2 instead of reading them
    VGen vg{};
    bool norm_sqrt = true;
    bool norm_accumulate = false;   // NORM: add the plain sum to *norm_out
    // Row-block partitions (multi-GPU): output rows [ra, rb) and rows [lo, hi]
    // that hold valid data (owned + ghost rows), all global row indices; the
    // field pointers are offset so that ptr + r*pitch is global row r.
    // rb < 0 means the whole level: ra = 0, rb = n+1, lo = 0, hi = n.
    int ra = 0, rb = -1, lo = 0, hi = -1;
    // prolongation passes on tiles only: the coarse level solved in the pass
    // (launch_smooth / launch_smooth_wpair return -4 when the pass would
    // march instead)
    CoarseFuse cf{};
};
int launch_smooth(const SmoothArgs &a, int sweeps, int mode, hipStream_t s);
// A W-cycle's post-smoothing of one visit + pre-smoothing of the next on a tile
// level as one pass (prolongation+add, 2 nsmooth sweeps, restriction); -1 if
// the level marches or nsmooth is not 1..3.
int launch_smooth_wpair(const SmoothArgs &a, int nsmooth, hipStream_t s);
// whether launch_smooth(a, sweeps, mode) generates v1, v2 (a.vg, the 3-sweep
// pre / post wave marches) instead of reading them: the launch's byte count
bool smooth_generates_velocity(const SmoothArgs &a, int sweeps, int mode);

// Cross-cycle fused finest-level pass (k_xsmooth): post-smoothing of cycle k
// (u_in + P(uc), `sweeps` sweeps, residual norm -> *norm_out as sqrt) into
// upost, and the pre-smoothing of cycle k+1 (`sweeps` sweeps, residual
// restricted into rhsc) into upre.  sweeps 2 or 3; returns the partials count
// or -1.  A row block [ra, rb) needs its rows [ra-14, rb+14) valid in the
// inputs (the pass's cone) and the matching coarse rows.
struct XArgs {
    const double *uin = nullptr;
    double *upost = nullptr, *upre = nullptr;
    const double *rhs = nullptr, *v1 = nullptr, *v2 = nullptr;
    const double *uc = nullptr;
    long pitchc = 0;
    double *rhsc = nullptr;
    double *partials = nullptr, *norm_out = nullptr;
    long n = 0, pitch = 0;
    Coef c{};
    bool store_post = true;   // false: u_post only feeds the norm (not the last cycle)
    bool norm_sqrt = true;    // false: *norm_out = sum of squares (multi-GPU partial)
    bool norm_accumulate = false;   // *norm_out += sum of squares (split pass)
    int ra = 0, rb = -1, lo = 0, hi = -1;   // row block (rb < 0: whole level), as SmoothArgs
    int min_rows = 64;   // fewest rows per workgroup (short bands: smaller, more parallel)
    // time-step mode (whole level, one GPU): B's pre-smoothing is the next time
    // step's, with its rhs formed from u_post into rhs_next and its initial
    // norm into *norm2_out; partials needs 2 * norm_partials_size() doubles
    double *rhs_next = nullptr, *norm2_out = nullptr;
    // separable velocity (sepvel.h): v1[R][c] = sa1[R] * sb1[c] exactly (global
    // row R, column c; sb zero-padded to the pitch), v2 likewise; all four set
    // = the pass reads rhs and u only (the 2-D v1 / v2 are not touched)
    const double *sa1 = nullptr, *sb1 = nullptr, *sa2 = nullptr, *sb2 = nullptr;
    // Split pass (the overlapped ghost exchange of a row block): band > 0 moves
    // rows [ra, ra+band) and [rb-band, rb) from the unguarded interior march to
    // the edge launch; phase 1 = the interior march only (returns its partials
    // count, no norm), phase 2 = the edge launch only, its partials written
    // after the first `partials_done` and the norm taken over both; 0 = both.
    int band = 0, phase = 0, partials_done = 0;
};
int launch_xsmooth(const XArgs &a, int sweeps, hipStream_t s);
// whether launch_xsmooth supports rhs_next on a whole level of size n
bool xstep_supported(long n);
// Cross pass: 1 = interior strips run the unguarded march (default), 0 = all guarded.
void set_xfast(long v);
long get_xfast();
void set_march_tile_rows(long v);
long get_march_tile_rows();
// Cross pass on row blocks of <= xtile_max_rows rows (default 4097): edges as
// LDS tiles instead of the guarded march (0 = never).
void set_xtile_max_rows(long v);
long get_xtile_max_rows();
// Levels with n <= tile_max_n use the 2-D tile form of the fused pass (small
// levels: latency bound), larger ones the row march.  Default 1024.
void set_tile_max_n(long v);
long get_tile_max_n();
// K = 3 tile passes on levels n >= tile32_min_n use 32 x 64 output tiles
// (default 2048), others 16 x 64; tile_xcd = 1 (default) deals the tiles
// XCD-contiguous.
void set_tile32_min_n(long v);
long get_tile32_min_n();
void set_tile_xcd(long v);
long get_tile_xcd();
// Row-march work order: bit 0 = band-major (neighbouring strip groups march
// the same rows together; launches of >= 192 rows per workgroup), bit 1 =
// XCD-contiguous workgroup order.  Default 3.
void set_march_order(long v);
long get_march_order();
// Fewest rows per workgroup of a wave-march launch (default 64): fewer,
// longer segments amortise the warm-up rows, more keep more waves in flight.
void set_march_min_rows(long v);
long get_march_min_rows();
// 1 (default): a march whose last band would be short runs one full-height
// segment per workgroup instead (partitioned levels); 0 = equal units only.
void set_march_seg(long v);
long get_march_seg();
// One colour, in place (two launches make a sweep).  Reference for A/B timing.
void launch_gs_colour(double *u, const double *rhs, const double *v1, const double *v2,
                      long n, long pitch, Coef c, int colour, hipStream_t s);
// residual at the fine even-even interior points written straight into the
// coarse rhs: rhsc[I][J] = res(2I, 2J), 1<=I,J<=n/2-1 (residual + restriction,
// multigrid.cpp:73-75).  Coarse boundary untouched.
void launch_residual_restrict(const double *u, const double *rhs, const double *v1,
                              const double *v2, long n, long pitch, Coef c, double *rhsc,
                              long pitchc, hipStream_t s);
// residual + sum of squares (not stored): partial sums -> norm into *out.
// Rows restricted to [ra, rb) (default: all); take_sqrt = false stores the sum.
void launch_residual_norm(const double *u, const double *rhs, const double *v1,
                          const double *v2, long n, long pitch, Coef c, double *partials,
                          double *out, hipStream_t s, int ra = 0, int rb = -1,
                          bool take_sqrt = true);
// residual stored (interior) into res (tower layout).
void launch_residual(double *res, const double *u, const double *rhs, const double *v1,
                     const double *v2, long n, long pitch, Coef c, hipStream_t s);
// uf += P(uc), every fine point (multigrid.cpp:81-83), nc = coarse n.
void launch_prolong_add(double *uf, long pitchf, const double *uc, long pitchc, long nc,
                        hipStream_t s);
void launch_rhs(double *rhs, const double *u, const double *v1, const double *v2, long n,
                long pitch, Coef c, hipStream_t s, int ra = 0, int rb = -1);
// compute_rhs stored AND the residual norm against it (rows [ra, rb)), one
// pass; the norm is bitwise launch_residual_norm's on the new rhs.
void launch_rhs_norm(double *rhs, const double *u, const double *v1, const double *v2, long n,
                     long pitch, Coef c, double *partials, double *out, hipStream_t s,
                     int ra = 0, int rb = -1, bool take_sqrt = true);
// Coarsest-level solve in one workgroup: repeat {GS; residual; norm} while
// norm > tol and it < maxit (multigrid.cpp:58-65), in place on u.
// zero_first: u = 0 before the first sweep.  stats[0] += iterations,
// stats[1] = last norm.  reps: the whole solve `reps` times in a row (a
// W-cycle's `shape` visits of the coarsest level, multigrid.cpp:52) in one launch.
void launch_coarse_solve(double *u, const double *rhs, const double *v1, const double *v2,
                         long n, long pitch, Coef c, double tol, int maxit, bool zero_first,
                         double *stats, hipStream_t s, int reps = 1);
constexpr long kCoarseOneWgMaxN = 256;
// 1 (default): coarsest levels n <= 64 solve with u, rhs, v1, v2 in LDS.
void set_coarse_lds(long v);
long get_coarse_lds();

}  // namespace mgx
