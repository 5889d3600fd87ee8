// kernels.hip -- CDNA4 (gfx950) fp64 stencil kernels for the multigrid V-cycle.
//
// Memory-bound work (31 flop / 40 B per smoother point): no MFMA.
// Every kernel is built with -ffp-contract=off and evaluates the reference's
// expressions term by term (gs.cpp:44, :75, :130, :238-241), so each value is
// bitwise the value the serial reference computes.
//
// Wave = 64 lanes; tower-layout kernels give each lane one column pair
// (2c, 2c+1) so every row access is a 16-B-per-lane, 1-KiB-per-wave load.
#include "stencil.h"

#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace mgx {

long tower_pitch(long n) { return (n + 1 + 15) / 16 * 16; }

Coef make_coef(double k, double nu, double h, int fm) {
    Coef c{};
    c.rr = 0.5 * k / (h * h);            // gs.cpp:9-11
    c.nu = nu;
    c.h = h;
    c.dgs = 1.0 - 4.0 * c.rr * nu;       // gs.cpp:130 denominator, gs.cpp:75 diagonal
    c.drhs = 1.0 + 4.0 * c.rr * nu;      // gs.cpp:44
    c.rdgs = 1.0 / c.dgs;                // RN(1/d) for the Markstein division
    c.dsign = std::signbit(c.dgs) ? 0x80000000u : 0u;
    c.g = c.rr / c.dgs;
    c.gn = c.g * nu;
    c.c2 = -2.0 * c.gn;
    c.fm = fm ? 1 : 0;
    return c;
}


namespace {

__global__ __launch_bounds__(kFinalThreads) void k_norm_final(const double *partials,
                                                              int count, double *out,
                                                              int take_sqrt = 1) {
    __shared__ double lds[16];
    double acc = 0.0;
    for (int i = threadIdx.x; i < count; i += kFinalThreads) acc += partials[i];
    double tot = block_sum(acc, lds);
    // take_sqrt: 1 = sqrt of the sum, 0 = the sum, 2 = add the sum to out[0]
    // (a pass split into several launches on one stream, multi-GPU partials)
    if (threadIdx.x == 0) out[0] = take_sqrt == 1 ? sqrt(tot) : take_sqrt == 2 ? out[0] + tot : tot;
}

// ============================================================ reference layout
// One lane per point, pitch n+1.  These back the gs.h-mirror entry points.
// 64-bit indexing throughout: at N = 65536 an array holds 4.3e9 elements
// (where the reference's int index math overflows).  Rows go over
// blockIdx.y with a grid stride (gridDim.y is capped at kMaxGridY).
constexpr long kMaxGridY = 32768;

__global__ __launch_bounds__(256) void k_raw_gs_colour(double *u, const double *rhs,
                                                       const double *v1, const double *v2,
                                                       long n, Coef c, int colour) {
    const long w = n + 1;
    for (long i = 1 + blockIdx.y; i < n; i += gridDim.y) {
        // points of this colour in row i: j = j0, j0+2, ... (gs.cpp:121-184)
        const long j0 = (colour == 0) ? (2 - (i & 1)) : (1 + (i & 1));
        const long j = j0 + 2 * ((long)blockIdx.x * blockDim.x + threadIdx.x);
        if (j >= n) continue;
        const long p = i * w + j;
        u[p] = gs_point(rhs[p], v1[p], v2[p], u[p - w], u[p - 1], u[p + w], u[p + 1], c);
    }
}

__global__ __launch_bounds__(256) void k_raw_residual(double *res, const double *u,
                                                      const double *rhs, const double *v1,
                                                      const double *v2, long n, Coef c) {
    const long w = n + 1;
    const long j = 1 + (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    for (long i = 1 + blockIdx.y; i < n; i += gridDim.y) {
        const long p = i * w + j;
        res[p] = res_point(rhs[p], v1[p], v2[p], u[p], u[p - w], u[p - 1], u[p + w], u[p + 1],
                           c);
    }
}

__global__ __launch_bounds__(256) void k_raw_rhs(double *rhs, const double *u,
                                                 const double *v1, const double *v2, long n,
                                                 Coef c) {
    const long w = n + 1;
    const long j = 1 + (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    for (long i = 1 + blockIdx.y; i < n; i += gridDim.y) {
        const long p = i * w + j;
        rhs[p] = rhs_point(v1[p], v2[p], u[p], u[p - w], u[p - 1], u[p + w], u[p + 1], c);
    }
}

// Fine point (I,J) of the (2n+1)^2 output from coarse (i,j)=(I/2,J/2) by the
// parity of (I,J) -- the same four formulas as gs.cpp:238-241 (their border
// variants gs.cpp:254-265 are the same expressions at i=n or j=n).
__device__ __forceinline__ double prolong_value(const double *u, long w, long I, long J) {
    const long i = I >> 1, j = J >> 1;
    const double *r0 = u + i * w + j;
    if (!(I & 1)) {
        if (!(J & 1)) return r0[0];
        return (r0[0] + r0[1]) / 2;
    }
    const double *r1 = r0 + w;
    if (!(J & 1)) return (r0[0] + r1[0]) / 2;
    return (r0[0] + r1[0] + r0[1] + r1[1]) / 4;
}

__global__ __launch_bounds__(256) void k_raw_prolongation(double *up, const double *u,
                                                          long n) {
    const long W = 2 * n + 1;
    const long J = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (J >= W) return;
    for (long I = blockIdx.y; I < W; I += gridDim.y) up[I * W + J] = prolong_value(u, n + 1, I, J);
}

// Injection of a block of coarse rows: dst row I, col J <- src row 2I, col 2J
// (restriction, gs.cpp:283; the tower build, multigrid.cpp:148-160).
__global__ __launch_bounds__(256) void k_injection_rows(double *dst, long dpitch,
                                                        const double *src, long spitch,
                                                        long rows, long cols) {
    const long J = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (J >= cols) return;
    for (long I = blockIdx.y; I < rows; I += gridDim.y)
        dst[I * dpitch + J] = src[2 * I * spitch + 2 * J];
}

__global__ __launch_bounds__(256) void k_row_nonzero(const double *v, long pitch, long n,
                                                     int *flags) {
    __shared__ int any;
    if (threadIdx.x == 0) any = 0;
    __syncthreads();
    const double *row = v + (long)blockIdx.x * pitch;
    int mine = 0;
    for (long j = threadIdx.x; j <= n; j += 256) mine |= row[j] != 0.0;
    if (mine) any = 1;   // benign: every writer stores 1
    __syncthreads();
    if (threadIdx.x == 0) flags[blockIdx.x] = any;
}

// Level g.l entry (i = blockIdx.y, j) against the generator (stencil.h
// vg_col): the same operands the wave march multiplies, compared bit for bit
__global__ __launch_bounds__(256) void k_vgen_check(const double *v1, const double *v2, int n,
                                                    long pitch, VGen g, int *ok, int r0, int r1) {
    const int j = blockIdx.x * 256 + threadIdx.x, N = n << g.l;
    if (j > n) return;
    const VGCol k = vg_col(j, n, g.l, g.strided);
    for (int i = r0 + (int)blockIdx.y; i <= r1; i += (int)gridDim.y) {
        const int st = vg_state(k, i), I = vg_row(k, i, st, g.l, N);
        if (I < 0 || I > N + 1) {
            *ok = 0;
            return;
        }
        const int c = st == 1 ? k.clo : k.chi;
        const double2 a = g.a[I];
        const double x = a.x * (st == 2 ? 0.0 : g.b1[c]), y = a.y * (st == 2 ? 0.0 : g.b2[c]);
        const long o = (long)i * pitch + j;
        if (__double_as_longlong(x) != __double_as_longlong(v1[o]) ||
            __double_as_longlong(y) != __double_as_longlong(v2[o]))
            *ok = 0;   // benign: every writer stores 0
    }
}

__global__ __launch_bounds__(256) void k_vgen_fill_rows(double2 *a, const double *v1,
                                                        const double *v2, long pitch, int l,
                                                        int js1, int js2, int r0, int r1) {
    const int i = r0 + (int)(blockIdx.x * 256 + threadIdx.x);
    if (i > r1) return;
    a[(long)i << l] = make_double2(v1[(long)i * pitch + js1], v2[(long)i * pitch + js2]);
}

// Interior sum of squares, rows split over the grid; deterministic per block.
__global__ __launch_bounds__(256) void k_norm_partial(const double *res, long n, long pitch,
                                                      int rows_per_block, double *partials) {
    __shared__ double lds[4];
    double acc = 0.0;
    const long i0 = 1 + (long)blockIdx.x * rows_per_block;
    const long i1 = std::min<long>(n, i0 + rows_per_block);
    for (long i = i0; i < i1; ++i)
        for (long j = 1 + threadIdx.x; j < n; j += 256) {
            const double r = res[i * pitch + j];
            acc += r * r;
        }
    double tot = block_sum(acc, lds);
    if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

// ================================================================ tower layout
//
// k_gs_sweep: one full red-black sweep in ONE pass over HBM.
//
// A workgroup owns a strip of W = 2*BLOCK columns [j0, j0+W) and a chunk of
// rows [a, b).  It marches down the rows keeping an 8-row ring of u in LDS
// (2 halo columns each side).  At step s it
//   - stores the prefetched u row s+3 into the ring,
//   - updates the RED points of row s+1 (they read only old BLACK values of
//     rows s..s+2), in the strip and in the 1-column halo,
//   - updates the BLACK points of row s-1 (they read only the NEW red values of
//     rows s-2..s, all final) and writes row s-1 to uout,
// with one barrier per step.  The red and black phases of a step touch
// disjoint ring entries, so they need no barrier between them.
// Red points of the halo columns and of row a-1 are recomputed from old
// values exactly as the neighbouring workgroup computes them, so the result
// is bitwise the in-place two-colour sweep of gs.cpp:109-189.  uout != uin:
// a workgroup's halo reads of uin must not see its neighbours' writes.
//
// HBM traffic per point: u read + rhs, v1, v2 read + u write = 40 B (the
// two-colour form reads every line twice: ~72-80 B).
template <int BLOCK>
struct SweepGeom {
    static constexpr int W = 2 * BLOCK;
    static constexpr int LW = W + 8;   // LDS row: x = col - j0 + 4
    static constexpr int RING = 8;
};

struct RowRV {           // rhs / v1 / v2 of one row at this lane's pair (+ halo col)
    double2 r, x, y;
    double hr, hx, hy;
};
struct Blk {             // black-point rhs / v1 / v2 kept for the black phase
    double r, x, y;
};

template <int BLOCK, bool ZERO_IN>
__global__ __launch_bounds__(BLOCK) void k_gs_sweep(const double *__restrict__ uin,
                                                    double *__restrict__ uout,
                                                    const double *__restrict__ rhs,
                                                    const double *__restrict__ v1,
                                                    const double *__restrict__ v2, int n,
                                                    long pitch, int chunk_rows, Coef c) {
    using G = SweepGeom<BLOCK>;
    __shared__ __attribute__((aligned(16))) double su[G::RING][G::LW];

    const int t = threadIdx.x;
    const long j0 = (long)blockIdx.x * G::W;
    const int a = blockIdx.y * chunk_rows;
    const int b = min(a + chunk_rows, n + 1);
    const long c0 = j0 + 2 * t;
    const bool act = c0 <= n;
    const int x0 = 2 * t + 4;
    // halo pairs: lane 0 loads cols (j0-2, j0-1) -> x 2,3; the last lane loads
    // cols (j0+W, j0+W+1) -> x W+4, W+5.
    const bool hl = (t == 0) && (j0 >= 2);
    const bool hr = (t == BLOCK - 1) && (j0 + G::W <= n);
    const long hlc = j0 - 2, hrc = j0 + G::W;

    auto in_rows = [&](int r) { return r >= 0 && r <= n; };

    // --- loaders
    auto load_u = [&](int r, double2 &own, double2 &hal) {
        if (ZERO_IN || !in_rows(r)) return;
        const double *row = uin + (long)r * pitch;
        if (act) own = ld2(row + c0);
        if (hl) hal = ld2(row + hlc);
        if (hr) hal = ld2(row + hrc);
    };
    auto put_u = [&](int r, const double2 &own, const double2 &hal) {
        double *s = su[r & (G::RING - 1)];
        const double2 z = make_double2(0.0, 0.0);
        if (act) st2(s + x0, ZERO_IN ? z : own);
        if (hl) st2(s + 2, ZERO_IN ? z : hal);
        if (hr) st2(s + G::W + 4, ZERO_IN ? z : hal);
    };
    auto load_rv = [&](int r, RowRV &q) {
        if (!in_rows(r)) return;
        const long o = (long)r * pitch;
        if (act) {
            q.r = ld2(rhs + o + c0);
            q.x = ld2(v1 + o + c0);
            q.y = ld2(v2 + o + c0);
        }
        if (hl) {
            q.hr = rhs[o + j0 - 1];
            q.hx = v1[o + j0 - 1];
            q.hy = v2[o + j0 - 1];
        }
        if (hr) {
            q.hr = rhs[o + hrc];
            q.hx = v1[o + hrc];
            q.hy = v2[o + hrc];
        }
    };

    // --- red phase: row r (its rhs/v in q)
    auto red = [&](int r, const RowRV &q) {
        if (r < 1 || r > n - 1) return;
        double *sm = su[r & 7], *sn = su[(r - 1) & 7], *ss = su[(r + 1) & 7];
        const int rs = r & 1;   // red column in my pair: c0 + rs
        const long col = c0 + rs;
        if (act && col >= 1 && col <= n - 1) {
            const int x = x0 + rs;
            sm[x] = gs_point(sel(q.r, rs), sel(q.x, rs), sel(q.y, rs), sn[x], sm[x - 1], ss[x],
                             sm[x + 1], c);
        }
        if (hl && rs == 1) {      // col j0-1 is red iff r odd
            sm[3] = gs_point(q.hr, q.hx, q.hy, sn[3], sm[2], ss[3], sm[4], c);
        }
        if (hr && rs == 0 && hrc <= n - 1) {   // col j0+W is red iff r even
            const int x = G::W + 4;
            sm[x] = gs_point(q.hr, q.hx, q.hy, sn[x], sm[x - 1], ss[x], sm[x + 1], c);
        }
    };
    // --- black phase + store: row q (its black-point rhs/v in k)
    auto black_store = [&](int r, const Blk &k) {
        if (r < a || r >= b || !act) return;
        double *sm = su[r & 7];
        double2 out = ld2(sm + x0);
        if (r >= 1 && r <= n - 1) {
            const int bs = 1 - (r & 1);
            const long col = c0 + bs;
            if (col >= 1 && col <= n - 1) {
                const int x = x0 + bs;
                const double v = gs_point(k.r, k.x, k.y, su[(r - 1) & 7][x], sm[x - 1],
                                          su[(r + 1) & 7][x], sm[x + 1], c);
                if (bs) out.y = v; else out.x = v;
            }
        }
        st2(uout + (long)r * pitch + c0, out);
    };
    auto keep_black = [&](int r, const RowRV &q, Blk &k) {
        const int bs = 1 - (r & 1);
        k.r = sel(q.r, bs);
        k.x = sel(q.x, bs);
        k.y = sel(q.y, bs);
    };

    // --- prologue: ring rows a-2, a-1, a; prefetch u row a+1, rhs/v row a-1.
    // Two named register sets (A/B) alternate between steps so that every
    // register index is static (no scratch).
    const double2 z2 = make_double2(0.0, 0.0);
    RowRV rvA{z2, z2, z2, 0.0, 0.0, 0.0}, rvB{z2, z2, z2, 0.0, 0.0, 0.0};
    Blk bkA{0.0, 0.0, 0.0}, bkB{0.0, 0.0, 0.0};
    double2 uoA = z2, uoB = z2, uhA = z2, uhB = z2;
    for (int r = a - 2; r <= a; ++r) {
        double2 o = z2, h = z2;
        load_u(r, o, h);
        put_u(r, o, h);
    }
    load_u(a + 1, uoB, uhB);
    load_rv(a - 1, rvB);
    __syncthreads();

#define MGX_GS_STEP(s, RCUR, RNXT, UCO, UCH, UNO, UNH, KB) \
    do {                                                  \
        put_u((s) + 3, UCO, UCH);                         \
        load_u((s) + 4, UNO, UNH);                        \
        load_rv((s) + 2, RNXT);                           \
        red((s) + 1, RCUR);                               \
        black_store((s) - 1, KB);                         \
        keep_black((s) + 1, RCUR, KB);                    \
        __syncthreads();                                  \
    } while (0)

    for (int s = a - 2; s <= b; s += 2) {
        MGX_GS_STEP(s, rvB, rvA, uoB, uhB, uoA, uhA, bkA);
        if (s + 1 > b) break;
        MGX_GS_STEP(s + 1, rvA, rvB, uoA, uhA, uoB, uhB, bkB);
    }
#undef MGX_GS_STEP
}

// One colour in place (two launches = one sweep).  Grid (strips, interior rows).
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_gs_colour(double *u, const double *rhs,
                                                     const double *v1, const double *v2,
                                                     int n, long pitch, Coef c, int colour) {
    const long i = 1 + blockIdx.y;
    const long c0 = (long)blockIdx.x * 2 * BLOCK + 2 * threadIdx.x;
    const int s = colour == 0 ? (int)(i & 1) : 1 - (int)(i & 1);
    const long col = c0 + s;
    if (col < 1 || col > n - 1) return;
    const long p = i * pitch + col;
    u[p] = gs_point(rhs[p], v1[p], v2[p], u[p - pitch], u[p - 1], u[p + pitch], u[p + 1], c);
}

// Row march for residual-type kernels.  MODE 0: sum of squares only; MODE 1:
// residual stored; MODE 2: compute_rhs stored; MODE 3: compute_rhs stored AND
// the sum of squares of the residual against it (a time step's rhs and
// mg_outer's initial norm, multigrid.cpp:104 after gs.cpp:24, in one pass:
// the same grid as MODE 0, so the partial sums and the norm are bitwise those
// of the two separate passes).  Block = 256 lanes = 512 cols,
// grid (strips, row groups); rows [1+g*R, min(n, 1+(g+1)*R)).
template <int MODE>
__global__ __launch_bounds__(256) void k_res_march(const double *__restrict__ u,
                                                   const double *__restrict__ rhs,
                                                   const double *__restrict__ v1,
                                                   const double *__restrict__ v2, int n,
                                                   long pitch, Coef c, int rows_per_group,
                                                   double *__restrict__ out,
                                                   double *__restrict__ partials, int r_first,
                                                   int r_end) {
    __shared__ double lds[4];
    const int t = threadIdx.x, lane = t & 63;
    const long c0 = (long)blockIdx.x * 512 + 2 * t;
    const bool act = c0 <= n;
    // interior rows [r_first, r_end) (a partition's owned rows, or 1..n-1)
    const long i0 = r_first + (long)blockIdx.y * rows_per_group;
    const long i1 = std::min<long>(r_end, i0 + rows_per_group);
    double acc = 0.0;
    const double2 z2 = make_double2(0.0, 0.0);
    double2 un = z2, um = z2, us = z2;
    if (act && i0 < i1) {
        un = ld2(u + (i0 - 1) * pitch + c0);
        um = ld2(u + i0 * pitch + c0);
    }
    for (long i = i0; i < i1; ++i) {
        const long o = i * pitch;
        double2 r2 = z2, x2 = z2, y2 = z2;
        if (act) {
            us = ld2(u + o + pitch + c0);
            if (MODE < 2) r2 = ld2(rhs + o + c0);
            x2 = ld2(v1 + o + c0);
            y2 = ld2(v2 + o + c0);
        }
        // west of c0 and east of c0+1 from the neighbouring lanes' pairs
        double w = __shfl_up(um.y, 1, 64);
        double e = __shfl_down(um.x, 1, 64);
        if (lane == 0 && act && c0 >= 1) w = u[o + c0 - 1];
        if (lane == 63 && act && c0 + 2 <= n) e = u[o + c0 + 2];
        if (act) {
            double2 res = z2;
            bool ok0 = c0 >= 1 && c0 <= n - 1, ok1 = c0 + 1 <= n - 1;
            if (MODE == 3) {
                // rhs (gs.cpp:44) stored, then the residual against it (:75)
                const double2 f = make_double2(rhs_point(x2.x, y2.x, um.x, un.x, w, us.x, um.y, c),
                                               rhs_point(x2.y, y2.y, um.y, un.y, um.x, us.y, e, c));
                if (ok0 && ok1) {
                    st2(out + o + c0, f);
                } else {
                    if (ok0) out[o + c0] = f.x;
                    if (ok1) out[o + c0 + 1] = f.y;
                }
                res.x = res_point(f.x, x2.x, y2.x, um.x, un.x, w, us.x, um.y, c);
                res.y = res_point(f.y, x2.y, y2.y, um.y, un.y, um.x, us.y, e, c);
            } else if (MODE == 2) {
                res.x = rhs_point(x2.x, y2.x, um.x, un.x, w, us.x, um.y, c);
                res.y = rhs_point(x2.y, y2.y, um.y, un.y, um.x, us.y, e, c);
            } else {
                res.x = res_point(r2.x, x2.x, y2.x, um.x, un.x, w, us.x, um.y, c);
                res.y = res_point(r2.y, x2.y, y2.y, um.y, un.y, um.x, us.y, e, c);
            }
            if (MODE == 0 || MODE == 3) {
                if (ok0) acc += res.x * res.x;
                if (ok1) acc += res.y * res.y;
            } else {
                if (ok0 && ok1) {
                    st2(out + o + c0, res);
                } else {
                    if (ok0) out[o + c0] = res.x;
                    if (ok1) out[o + c0 + 1] = res.y;
                }
            }
        }
        un = um;
        um = us;
    }
    if (MODE == 0 || MODE == 3) {
        double tot = block_sum(acc, lds);
        if (t == 0) partials[blockIdx.y * gridDim.x + blockIdx.x] = tot;
    }
}

// residual at fine (2I, 2J) -> rhsc[I][J], 1 <= I,J <= nc-1 (nc = n/2).
// One lane per coarse column; block 256 coarse columns; grid (strips, groups).
__global__ __launch_bounds__(256) void k_res_restrict(const double *__restrict__ u,
                                                      const double *__restrict__ rhs,
                                                      const double *__restrict__ v1,
                                                      const double *__restrict__ v2, int n,
                                                      long pitch, Coef c, double *rhsc,
                                                      long pitchc, int rows_per_group) {
    const int t = threadIdx.x, lane = t & 63;
    const long nc = n / 2;
    const long J = (long)blockIdx.x * 256 + t;
    const bool act = J >= 1 && J <= nc - 1;
    const long I0 = 1 + (long)blockIdx.y * rows_per_group;
    const long I1 = std::min<long>(nc, I0 + rows_per_group);
    const long fc = 2 * J;   // fine column
    const bool ld = J <= nc; // lanes whose pair (2J, 2J+1) exists
    double2 mid = make_double2(0.0, 0.0);
    double un = 0.0, us = 0.0;
    if (ld && I0 < I1) un = u[(2 * I0 - 1) * pitch + fc];
    for (long I = I0; I < I1; ++I) {
        const long o = 2 * I * pitch;
        double r = 0.0, x = 0.0, y = 0.0;
        if (ld) {
            mid = ld2(u + o + fc);
            us = u[o + pitch + fc];
        }
        if (act) {
            r = rhs[o + fc];
            x = v1[o + fc];
            y = v2[o + fc];
        }
        double w = __shfl_up(mid.y, 1, 64);   // u[2I][2J-1]
        if (lane == 0 && act) w = u[o + fc - 1];
        if (act) rhsc[I * pitchc + J] = res_point(r, x, y, mid.x, un, w, us, mid.y, c);
        un = us;   // fine row 2I+1 is the north row of coarse row I+1
    }
}

// uf += P(uc) on every fine point.  Lane = fine pair (2j, 2j+1) <- coarse j.
__global__ __launch_bounds__(256) void k_prolong_add(double *uf, long pitchf,
                                                     const double *uc, long pitchc, int nc) {
    const long I = blockIdx.y;   // fine row 0..2nc
    const long j = (long)blockIdx.x * 256 + threadIdx.x;
    if (j > nc) return;
    const long i = I >> 1;
    const double *r0 = uc + i * pitchc + j;
    double2 p;
    const bool has1 = j + 1 <= nc;
    if (!(I & 1)) {
        p.x = r0[0];
        p.y = has1 ? (r0[0] + r0[1]) / 2 : 0.0;
    } else {
        const double *r1 = r0 + pitchc;
        p.x = (r0[0] + r1[0]) / 2;
        p.y = has1 ? (r0[0] + r1[0] + r0[1] + r1[1]) / 4 : 0.0;
    }
    double *f = uf + I * pitchf + 2 * j;
    if (has1) {
        double2 v = ld2(f);
        v.x += p.x;
        v.y += p.y;
        st2(f, v);
    } else {
        f[0] += p.x;
    }
}

// Coarsest level in one workgroup (multigrid.cpp:55-65), in place.
// FM: fp_mode fma (stencil.h): the contracted update and residual.
template <bool FM>
__global__ __launch_bounds__(1024) void k_coarse_solve(double *u, const double *rhs,
                                                       const double *v1, const double *v2,
                                                       int n, long pitch, Coef c, double tol,
                                                       int maxit, int zero_first, int reps,
                                                       double *stats) {
    __shared__ double lds[16];
    __shared__ double s_norm;
    const int t = threadIdx.x;
    // 64 x 16 threads: lane tx walks the columns, ty the rows (no integer
    // division in the loops: 64-bit div/mod is a long emulated sequence)
    const int tx = t & 63, ty = t >> 6;
    const double hh = c.h * 0.5;   // FM: t = v*h/2
    if (zero_first) {
        for (long p = t; p < (long)(n + 1) * pitch; p += 1024) u[p] = 0.0;
        __syncthreads();
    }
    int total = 0;
    double res = 1.0;
    for (int rep = 0; rep < reps; ++rep) {
    int it = 0;
    res = 1.0;
    while (it < maxit && res > tol) {
        for (int colour = 0; colour < 2; ++colour) {
            for (int i = 1 + ty; i <= n - 1; i += 16) {
                // first column of this colour in row i: (i + j) & 1 == colour
                const int jc = 1 + ((i + 1 + colour) & 1);
                for (int j = jc + 2 * tx; j <= n - 1; j += 128) {
                    const long p = (long)i * pitch + j;
                    u[p] = FM ? fm_upd_t(rhs[p] * c.rdgs, v1[p] * hh, v2[p] * hh, u[p - pitch],
                                         u[p - 1], u[p + pitch], u[p + 1], c)
                              : gs_point(rhs[p], v1[p], v2[p], u[p - pitch], u[p - 1],
                                         u[p + pitch], u[p + 1], c);
                }
            }
            __syncthreads();
        }
        double acc = 0.0;
        for (int i = 1 + ty; i <= n - 1; i += 16)
            for (int j = 1 + tx; j <= n - 1; j += 64) {
                const long p = (long)i * pitch + j;
                const double r = FM ? fm_res_t(rhs[p] * c.rdgs, v1[p] * hh, v2[p] * hh, u[p],
                                               u[p - pitch], u[p - 1], u[p + pitch], u[p + 1], c)
                                    : res_point(rhs[p], v1[p], v2[p], u[p], u[p - pitch],
                                                u[p - 1], u[p + pitch], u[p + 1], c);
                acc += r * r;
            }
        double s = block_sum(acc, lds);
        if (t == 0) s_norm = sqrt(s);
        __syncthreads();
        res = s_norm;
        ++it;
        __syncthreads();
    }
    total += it;
    }
    if (t == 0) {
        stats[0] += total;
        stats[1] = res;
    }
}

// k_coarse_solve_lds: the coarsest solve with u in LDS (n <= 64, stencil.h
// coarse_lds_body), one workgroup.
template <bool FM>
__global__ __launch_bounds__(1024) void k_coarse_solve_lds(double *u, const double *rhs,
                                                           const double *v1, const double *v2,
                                                           int n, long pitch, Coef c, double tol,
                                                           int maxit, int zero_first, int reps,
                                                           double *stats) {
    __shared__ double su[kCoarseLdsNP * kCoarseLdsNP];
    __shared__ double lds[16];
    __shared__ double s_norm;
    coarse_lds_body<FM>(su, lds, &s_norm, u, rhs, v1, v2, n, pitch, c, tol, maxit, zero_first,
                        reps, stats, true);
}

}  // namespace

// ------------------------------------------------------------------ launchers
static unsigned grid_y(long rows) { return (unsigned)std::max<long>(1, std::min(rows, kMaxGridY)); }

void launch_raw_gs_colour(double *u, const double *rhs, const double *v1, const double *v2,
                          long n, Coef c, int colour, hipStream_t s) {
    if (n < 2) return;
    dim3 g(cdiv(n / 2, 256), grid_y(n - 1));
    MGX_LAUNCH(k_raw_gs_colour, g, dim3(256), s, u, rhs, v1, v2, n, c, colour);
}
void launch_raw_residual(double *res, const double *u, const double *rhs, const double *v1,
                         const double *v2, long n, Coef c, hipStream_t s) {
    if (n < 2) return;
    dim3 g(cdiv(n - 1, 256), grid_y(n - 1));
    MGX_LAUNCH(k_raw_residual, g, dim3(256), s, res, u, rhs, v1, v2, n, c);
}
void launch_raw_rhs(double *rhs, const double *u, const double *v1, const double *v2, long n,
                    Coef c, hipStream_t s) {
    if (n < 2) return;
    dim3 g(cdiv(n - 1, 256), grid_y(n - 1));
    MGX_LAUNCH(k_raw_rhs, g, dim3(256), s, rhs, u, v1, v2, n, c);
}
void launch_raw_prolongation(double *up, const double *u, long n, hipStream_t s) {
    const long W = 2 * n + 1;
    dim3 g(cdiv(W, 256), grid_y(W));
    MGX_LAUNCH(k_raw_prolongation, g, dim3(256), s, up, u, n);
}
void launch_injection(double *dst, long dst_pitch, const double *src, long src_pitch, long m,
                      hipStream_t s) {
    launch_injection_rows(dst, dst_pitch, src, src_pitch, m, m, s);
}

void launch_injection_rows(double *dst, long dst_pitch, const double *src, long src_pitch,
                           long rows, long cols, hipStream_t s) {
    if (rows <= 0 || cols <= 0) return;
    dim3 g(cdiv(cols, 256), grid_y(rows));
    MGX_LAUNCH(k_injection_rows, g, dim3(256), s, dst, dst_pitch, src, src_pitch, rows, cols);
}

void launch_row_nonzero(const double *v, long pitch, long n, int *flags, hipStream_t s) {
    MGX_LAUNCH(k_row_nonzero, dim3((unsigned)(n + 1)), dim3(256), s, v, pitch, n, flags);
}

void launch_vgen_check(const double *v1, const double *v2, long n, long pitch, VGen g, int *ok,
                       hipStream_t s, int r0, int r1) {
    if (r1 < 0) {
        r0 = 0;
        r1 = (int)n;
    }
    if (r1 < r0) return;
    const unsigned rows = (unsigned)std::min<long>(r1 - r0 + 1, 4096);
    MGX_LAUNCH(k_vgen_check, dim3((unsigned)((n + 256) / 256), rows), dim3(256), s, v1, v2, (int)n,
               pitch, g, ok, r0, r1);
}

void launch_vgen_fill_rows(double2 *a, const double *v1, const double *v2, long pitch, int l,
                           int js1, int js2, int r0, int r1, hipStream_t s) {
    if (r1 < r0) return;
    MGX_LAUNCH(k_vgen_fill_rows, dim3((unsigned)((r1 - r0 + 256) / 256)), dim3(256), s, a, v1, v2,
               pitch, l, js1, js2, r0, r1);
}

int norm_partials_size() { return kNormBlocks; }

void launch_norm(const double *res, long n, long pitch, double *partials, double *out,
                 hipStream_t s) {
    const long rows = std::max<long>(n - 1, 0);
    int rpb = (int)std::max<long>(1, (rows + 2047) / 2048);
    int blocks = (int)std::max<long>(1, (rows + rpb - 1) / rpb);
    MGX_LAUNCH(k_norm_partial, dim3(blocks), dim3(256), s, res, n, pitch, rpb, partials);
    MGX_LAUNCH(k_norm_final, dim3(1), dim3(kFinalThreads), s, (const double *)partials, blocks,
               out);
}

void launch_gs_sweep(const double *uin, double *uout, const double *rhs, const double *v1,
                     const double *v2, long n, long pitch, Coef c, bool zero_in,
                     hipStream_t s) {
    // Wide strips for big levels; narrow strips keep mid-size levels parallel.
    if (n >= 4096) {
        constexpr int B = 256;
        const unsigned strips = cdiv(n + 1, 2 * B);
        int R = 256;
        dim3 g(strips, cdiv(n + 1, R));
        if (zero_in)
            MGX_LAUNCH((k_gs_sweep<B, true>), g, dim3(B), s, uin, uout, rhs, v1, v2, (int)n,
                       pitch, R, c);
        else
            MGX_LAUNCH((k_gs_sweep<B, false>), g, dim3(B), s, uin, uout, rhs, v1, v2, (int)n,
                       pitch, R, c);
    } else {
        constexpr int B = 64;
        const unsigned strips = cdiv(n + 1, 2 * B);
        // aim at >= ~1024 workgroups, chunks of 16..256 rows
        long want = std::max<long>(1, 1024 / (long)strips);
        int R = (int)std::min<long>(256, std::max<long>(16, (n + 1 + want - 1) / want));
        dim3 g(strips, cdiv(n + 1, R));
        if (zero_in)
            MGX_LAUNCH((k_gs_sweep<B, true>), g, dim3(B), s, uin, uout, rhs, v1, v2, (int)n,
                       pitch, R, c);
        else
            MGX_LAUNCH((k_gs_sweep<B, false>), g, dim3(B), s, uin, uout, rhs, v1, v2, (int)n,
                       pitch, R, c);
    }
}

void launch_norm_final(const double *partials, int count, double *out, int mode,
                       hipStream_t s) {
    MGX_LAUNCH(k_norm_final, dim3(1), dim3(kFinalThreads), s, partials, count, out, mode);
}

long g_march_min_rows = 32;   // fewest rows per workgroup of a wave march (tuning key)
void set_march_min_rows(long v) { g_march_min_rows = v; }
long get_march_min_rows() { return g_march_min_rows; }

long g_march_order = 3;   // tuning key "march_order": bit 0 bands, bit 1 XCD order
static long march_order() { return g_march_order; }
void set_march_order(long v) { g_march_order = v; }
long get_march_order() { return g_march_order; }

// The work order of a launch of `upw` units per workgroup (march_order):
// band-major with bands of upw rows on a one-region launch, and/or the
// XCD-contiguous workgroup order.  Only the order changes, not the work.
// Measured (N=16384, per cycle): cross pass 2.92 -> 2.78 ms, level 1 1.13 ->
// 1.11 ms; with ~80-row segments (level 2) bands cost +12 %, so they apply
// from kBandMinRows rows per workgroup.
constexpr long kBandMinRows = 192;
MarchRegions order_regions(const MarchRegions &reg, long upw) {
    MarchRegions r = reg;
    const long m = march_order();
    if ((m & 1) && r.count == 1 && upw >= kBandMinRows && upw < r.r1[0] - r.r0[0])
        r.band[0] = (int)upw;
    if (m & 2) r.xcd = 1;
    return r;
}

long g_march_seg = 1;   // tuning key "march_seg"
void set_march_seg(long v) { g_march_seg = v; }
long get_march_seg() { return g_march_seg; }

// Work plan of a march launch over `reg`: workgroups, units per workgroup and
// the ordered regions.  Equal units per workgroup, band-major -- except that
// when the last band is short (a row block of a partitioned level: 2048 rows
// in bands of 328) its workgroups would each march pieces of several groups,
// every piece paying the warm-up of ~`warm` rows; then k full-height bands of
// one segment per workgroup (seg) when that gives the shorter longest march
// (level 0 at G=8: 492 -> 382 steps).
unsigned plan_march(const MarchRegions &reg, int wpb, long slots, long min_rows,
                           long max_wgs, int warm, long &upw, MarchRegions &out) {
    const long total = reg.pre[reg.count];
    long g = std::max<long>(1, std::min<long>(slots, total / min_rows));
    g = std::min(g, max_wgs);
    upw = (total + g - 1) / g;
    unsigned grid = (unsigned)((total + upw - 1) / upw);
    out = order_regions(reg, upw);
    if (!g_march_seg || out.count != 1 || out.band[0] <= 0) return grid;
    const long rows = out.r1[0] - out.r0[0];
    const long ng = (out.slim[0] - out.sfirst[0] + wpb - 1) / wpb;
    const long hl = rows % upw;   // height of the last band
    if (hl == 0) return grid;
    const long cur = upw + ((upw + hl - 1) / hl) * warm;   // its longest march
    const long k = std::min(slots, max_wgs) / ng;          // bands of one segment each
    if (k < 1) return grid;
    const long B = (rows + k - 1) / k;
    if (B + warm >= cur) return grid;
    out.band[0] = (int)B;
    out.seg = 1;
    upw = B;
    return (unsigned)(ng * ((rows + B - 1) / B));
}

void launch_gs_colour(double *u, const double *rhs, const double *v1, const double *v2,
                      long n, long pitch, Coef c, int colour, hipStream_t s) {
    if (n < 2) return;
    constexpr int B = 256;
    dim3 g(cdiv(n + 1, 2 * B), (unsigned)(n - 1));
    MGX_LAUNCH((k_gs_colour<B>), g, dim3(B), s, u, rhs, v1, v2, (int)n, pitch, c, colour);
}

static void res_grid(long n, long rows, dim3 &g, int &R) {
    const unsigned strips = cdiv(n + 1, 512);
    rows = std::max<long>(rows, 1);
    long want = std::max<long>(1, 4096 / (long)strips);
    R = (int)std::max<long>(8, (rows + want - 1) / want);
    g = dim3(strips, cdiv(rows, R));
}

static void interior_rows(long n, int ra, int rb, int &f, int &e) {
    if (rb < 0) {
        ra = 0;
        rb = (int)n + 1;
    }
    f = std::max(1, ra);
    e = std::min((int)n, rb);
}

void launch_residual_norm(const double *u, const double *rhs, const double *v1,
                          const double *v2, long n, long pitch, Coef c, double *partials,
                          double *out, hipStream_t s, int ra, int rb, bool take_sqrt) {
    int f, e;
    interior_rows(n, ra, rb, f, e);
    dim3 g;
    int R;
    res_grid(n, e - f, g, R);
    MGX_LAUNCH((k_res_march<0>), g, dim3(256), s, u, rhs, v1, v2, (int)n, pitch, c, R,
               (double *)nullptr, partials, f, e);
    MGX_LAUNCH(k_norm_final, dim3(1), dim3(kFinalThreads), s, (const double *)partials,
               (int)(g.x * g.y), out, take_sqrt ? 1 : 0);
}

void launch_residual(double *res, const double *u, const double *rhs, const double *v1,
                     const double *v2, long n, long pitch, Coef c, hipStream_t s) {
    int f, e;
    interior_rows(n, 0, -1, f, e);
    dim3 g;
    int R;
    res_grid(n, e - f, g, R);
    MGX_LAUNCH((k_res_march<1>), g, dim3(256), s, u, rhs, v1, v2, (int)n, pitch, c, R, res,
               (double *)nullptr, f, e);
}

void launch_rhs(double *rhs, const double *u, const double *v1, const double *v2, long n,
                long pitch, Coef c, hipStream_t s, int ra, int rb) {
    int f, e;
    interior_rows(n, ra, rb, f, e);
    dim3 g;
    int R;
    res_grid(n, e - f, g, R);
    MGX_LAUNCH((k_res_march<2>), g, dim3(256), s, u, (const double *)nullptr, v1, v2, (int)n,
               pitch, c, R, rhs, (double *)nullptr, f, e);
}

void launch_rhs_norm(double *rhs, const double *u, const double *v1, const double *v2, long n,
                     long pitch, Coef c, double *partials, double *out, hipStream_t s, int ra,
                     int rb, bool take_sqrt) {
    int f, e;
    interior_rows(n, ra, rb, f, e);
    dim3 g;
    int R;
    res_grid(n, e - f, g, R);
    MGX_LAUNCH((k_res_march<3>), g, dim3(256), s, u, (const double *)nullptr, v1, v2, (int)n,
               pitch, c, R, rhs, partials, f, e);
    MGX_LAUNCH(k_norm_final, dim3(1), dim3(kFinalThreads), s, (const double *)partials,
               (int)(g.x * g.y), out, take_sqrt ? 1 : 0);
}

void launch_residual_restrict(const double *u, const double *rhs, const double *v1,
                              const double *v2, long n, long pitch, Coef c, double *rhsc,
                              long pitchc, hipStream_t s) {
    const long nc = n / 2;
    if (nc < 2) return;
    const unsigned strips = cdiv(nc + 1, 256);
    const long rows = nc - 1;
    long want = std::max<long>(1, 4096 / (long)strips);
    int R = (int)std::max<long>(4, (rows + want - 1) / want);
    dim3 g(strips, cdiv(rows, R));
    MGX_LAUNCH(k_res_restrict, g, dim3(256), s, u, rhs, v1, v2, (int)n, pitch, c, rhsc, pitchc,
               R);
}

void launch_prolong_add(double *uf, long pitchf, const double *uc, long pitchc, long nc,
                        hipStream_t s) {
    dim3 g(cdiv(nc + 1, 256), (unsigned)(2 * nc + 1));
    MGX_LAUNCH(k_prolong_add, g, dim3(256), s, uf, pitchf, uc, pitchc, (int)nc);
}

long g_coarse_lds = 1;   // tuning key "coarse_lds"
void set_coarse_lds(long v) { g_coarse_lds = v; }
long get_coarse_lds() { return g_coarse_lds; }

void launch_coarse_solve(double *u, const double *rhs, const double *v1, const double *v2,
                         long n, long pitch, Coef c, double tol, int maxit, bool zero_first,
                         double *stats, hipStream_t s, int reps) {
    const int zf = zero_first ? 1 : 0;
    if (n <= kCoarseLdsMaxN && g_coarse_lds) {
        if (c.fm)
            MGX_LAUNCH(k_coarse_solve_lds<true>, dim3(1), dim3(1024), s, u, rhs, v1, v2, (int)n,
                       pitch, c, tol, maxit, zf, reps, stats);
        else
            MGX_LAUNCH(k_coarse_solve_lds<false>, dim3(1), dim3(1024), s, u, rhs, v1, v2, (int)n,
                       pitch, c, tol, maxit, zf, reps, stats);
        return;
    }
    if (c.fm)
        MGX_LAUNCH(k_coarse_solve<true>, dim3(1), dim3(1024), s, u, rhs, v1, v2, (int)n, pitch, c,
                   tol, maxit, zf, reps, stats);
    else
        MGX_LAUNCH(k_coarse_solve<false>, dim3(1), dim3(1024), s, u, rhs, v1, v2, (int)n, pitch, c,
                   tol, maxit, zf, reps, stats);
}

// ---------------------------------------------------------------- probes
// Streaming-bandwidth probes (the practical HBM ceiling SURVEY 8d asks for
// beside the 8 TB/s spec): `nin` double2 input streams and one output stream,
// out[i] = sum of the inputs.  nin = 1 is a copy; nin = 4 is the smoother's
// stream shape (u, rhs, v1, v2 in, u out).  The access shape is the best one
// measured on the box (tools/probe/bw2.hip): one 16-B element per lane, one
// workgroup per 4 KiB, non-temporal loads and stores -- 6.6 TB/s copy, 6.1 TB/s
// 4-in/1-out, against 5.0-5.4 TB/s for grid-stride, per-workgroup chunks or
// column-strip marches of the same bytes.
template <int NIN>
__global__ __launch_bounds__(256) void k_stream(const double2 *__restrict__ a,
                                                const double2 *__restrict__ b,
                                                const double2 *__restrict__ c,
                                                const double2 *__restrict__ d,
                                                double2 *__restrict__ o, long n) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        double2 v = ld2s(reinterpret_cast<const double *>(a + i));
        if (NIN > 1) {
            const double2 y = ld2s(reinterpret_cast<const double *>(b + i));
            const double2 z = ld2s(reinterpret_cast<const double *>(c + i));
            const double2 w = ld2s(reinterpret_cast<const double *>(d + i));
            v.x += y.x + z.x + w.x;
            v.y += y.y + z.y + w.y;
        }
        st2s(reinterpret_cast<double *>(o + i), v);
    }
}

void launch_stream(const double *a, const double *b, const double *c, const double *d,
                   double *o, long n2, int nin, int grid, hipStream_t s) {
    if (nin == 1)
        MGX_LAUNCH(k_stream<1>, dim3(grid), dim3(256), s, (const double2 *)a, (const double2 *)b,
                   (const double2 *)c, (const double2 *)d, (double2 *)o, n2);
    else
        MGX_LAUNCH(k_stream<4>, dim3(grid), dim3(256), s, (const double2 *)a, (const double2 *)b,
                   (const double2 *)c, (const double2 *)d, (double2 *)o, n2);
}

}  // namespace mgx
