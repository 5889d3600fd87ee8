// kernels.hip -- CDNA4 (gfx950) fp64 stencil kernels for the multigrid V-cycle.
//
// Memory-bound work (31 flop / 40 B per smoother point): no MFMA.
// Every kernel is built with -ffp-contract=off and evaluates the reference's
// expressions term by term (gs.cpp:44, :75, :130, :238-241), so each value is
// bitwise the value the serial reference computes.
//
// Wave = 64 lanes; tower-layout kernels give each lane one column pair
// (2c, 2c+1) so every row access is a 16-B-per-lane, 1-KiB-per-wave load.
#include "kernels.h"

#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace mgx {

long tower_pitch(long n) {
    static long pad = -1;
    if (pad < 0) {
        const char *e = getenv("MGX_PITCH_PAD");
        pad = e ? std::max(0L, atol(e) / 16 * 16) : 0;
    }
    return (n + 1 + 15) / 16 * 16 + pad;
}

Coef make_coef(double k, double nu, double h) {
    Coef c;
    c.rr = 0.5 * k / (h * h);            // gs.cpp:9-11
    c.nu = nu;
    c.h = h;
    c.dgs = 1.0 - 4.0 * c.rr * nu;       // gs.cpp:130 denominator, gs.cpp:75 diagonal
    c.drhs = 1.0 + 4.0 * c.rr * nu;      // gs.cpp:44
    c.rdgs = 1.0 / c.dgs;                // RN(1/d) for the Markstein division
    c.dsign = std::signbit(c.dgs) ? 0x80000000u : 0u;
    return c;
}

namespace {

// ------------------------------------------------------------------ point math
// gs.cpp:14-20
__device__ __forceinline__ double coef_a(double v, const Coef &c) {
    return c.rr * (-v * c.h / 2.0 + c.nu);
}
__device__ __forceinline__ double coef_b(double v, const Coef &c) {
    return c.rr * (v * c.h / 2.0 + c.nu);
}
// gs.cpp:126-130: aa,bb from v2 (y-neighbours W/E), cc,dd from v1 (x-neighbours N/S)
__device__ __forceinline__ double gs_point(double rhs, double v1, double v2, double uN,
                                           double uW, double uS, double uE, const Coef &c) {
    const double aa = coef_a(v2, c), bb = coef_b(v2, c);
    const double cc = coef_a(v1, c), dd = coef_b(v1, c);
    return (rhs - cc * uN - aa * uW - dd * uS - bb * uE) / c.dgs;
}
// gs.cpp:75
__device__ __forceinline__ double res_point(double rhs, double v1, double v2, double u,
                                            double uN, double uW, double uS, double uE,
                                            const Coef &c) {
    const double aa = coef_a(v2, c), bb = coef_b(v2, c);
    const double cc = coef_a(v1, c), dd = coef_b(v1, c);
    return rhs - (c.dgs * u + cc * uN + aa * uW + dd * uS + bb * uE);
}
// gs.cpp:44
__device__ __forceinline__ double rhs_point(double v1, double v2, double u, double uN,
                                            double uW, double uS, double uE, const Coef &c) {
    const double aa = coef_a(v2, c), bb = coef_b(v2, c);
    const double cc = coef_a(v1, c), dd = coef_b(v1, c);
    return c.drhs * u - cc * uN - aa * uW - dd * uS - bb * uE;
}

__device__ __forceinline__ double2 ld2(const double *p) {
    return *reinterpret_cast<const double2 *>(p);
}
__device__ __forceinline__ void st2(double *p, double2 v) {
    *reinterpret_cast<double2 *>(p) = v;
}
// Streaming (non-temporal) forms for data touched once per pass: the fused
// smoother's rhs/v1/v2/u rows and its output rows.  MGX_NT=0 turns them into
// plain accesses (A/B builds).
#ifndef MGX_NT
#define MGX_NT 1
#endif
typedef double mgx_d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld2s(const double *p) {
#if MGX_NT
    const mgx_d2v v = __builtin_nontemporal_load(reinterpret_cast<const mgx_d2v *>(p));
    return make_double2(v.x, v.y);
#else
    return ld2(p);
#endif
}
__device__ __forceinline__ void st2s(double *p, double2 v) {
#if MGX_NT
    const mgx_d2v w = {v.x, v.y};
    __builtin_nontemporal_store(w, reinterpret_cast<mgx_d2v *>(p));
#else
    st2(p, v);
#endif
}
// Conditional stores of the march (exec-masked).  A hardware-dropped raw
// buffer store (offset past the row) would avoid the exec branch, but measured
// +20 % on the cross pass (3.25 vs 2.72 ms at N=16384), so these stay
// branches.  The u rows they write are next read a whole coarse descent or
// cycle later, so they are streaming stores (MGX_NTST): -1.7 % per V-cycle
// (level 0 -0.02 ms, level 1 -0.035 ms); the coarse rhs, read by the very next
// pass, stays a plain store.
#ifndef MGX_NTST
#define MGX_NTST 1
#endif
__device__ __forceinline__ void st2_if(double *row, int col, bool on, double2 v) {
#if MGX_NTST
    if (on) st2s(row + col, v);
#else
    if (on) st2(row + col, v);
#endif
}
__device__ __forceinline__ void st1_if(double *row, int col, bool on, double v) {
    if (on) row[col] = v;
}
// The same accesses as a uniform row base + a per-lane unsigned byte offset:
// the saddr form of global_load / global_store (SGPR base, 32-bit VGPR
// offset) instead of a 64-bit per-lane address -- no 64-bit address add per
// access, and the march keeps one offset register per column instead of a
// pointer pair per field.  (Lanes whose offset would be negative are never
// enabled: `on` implies an owned column.)
__device__ __forceinline__ const char *rowb(const double *row, unsigned boff) {
    return reinterpret_cast<const char *>(row) + boff;
}
__device__ __forceinline__ double2 ld2u(const double *row, unsigned boff) {
    return *reinterpret_cast<const double2 *>(rowb(row, boff));
}
__device__ __forceinline__ double ld1u(const double *row, unsigned boff) {
    return *reinterpret_cast<const double *>(rowb(row, boff));
}
__device__ __forceinline__ void st2_ifu(double *row, int col, bool on, double2 v) {
    double *p = reinterpret_cast<double *>(const_cast<char *>(rowb(row, (unsigned)col * 8u)));
#if MGX_NTST
    if (on) st2s(p, v);
#else
    if (on) st2(p, v);
#endif
}
__device__ __forceinline__ void st1_ifu(double *row, int col, bool on, double v) {
    double *p = reinterpret_cast<double *>(const_cast<char *>(rowb(row, (unsigned)col * 8u)));
    if (on) *p = v;
}
__device__ __forceinline__ double sel(double2 p, int s) {
    const double x = p.x, y = p.y;
    return s ? y : x;
}

// Wave-wide sum (64 lanes), fixed butterfly order -> deterministic.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
// Block-wide sum, result valid in thread 0.  blockDim.x multiple of 64, <= 1024.
__device__ __forceinline__ double block_sum(double v, double *lds) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) lds[w] = v;
    __syncthreads();
    double tot = 0.0;
    if (threadIdx.x == 0) {
        const int nw = blockDim.x >> 6;
        for (int i = 0; i < nw; ++i) tot += lds[i];
    }
    return tot;
}

constexpr int kNormBlocks = 8192;   // capacity of the partials buffer
constexpr int kFinalThreads = 1024;

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

// Temporal blocking, shared by the row marches (k_wsmooth, k_xsmooth) and
// the LDS tiles (k_smooth_tile): K red-black sweeps in ONE pass over HBM.
//
// The 2K half-sweeps are "stages" h = 0..S-1 (S = 2K; even h red, odd h
// black).  A march goes down the rows of a strip; at step s stage h
// updates its colour in row s+1-h, reading the other colour of rows
// s-h..s+2-h as left by stage h-1.  Each lane owns one column pair
// (2c, 2c+1).
// Optional last stage h = S (RESTRICT / NORM): the residual of row s+1-S,
// whose neighbours are final by then.
//
// Halo: the outer H lanes on each side own halo pairs that are loaded and
// updated like the strip but never stored.  Stage h is exact on a region that
// shrinks by one column (and one row) per stage, so after E stages (E = S,
// +1 with a residual stage, H = ceil(E/2)) the strip [j0, j0+W) and the rows
// [a, b) are exact; values outside that cone may be garbage and are never
// stored or read by exact values.  Every exact value is computed from exactly
// the operands the sequential gs.cpp:109-189 sweeps use, so the result is
// bitwise that of K reference sweeps.
//
// rhs / v1 / v2 of a row stay in registers from the step they are loaded to
// the last stage that needs them, in the ring slot that dies each step; u
// rows are prefetched ahead too (two alternating register sets).  The step
// loop is unrolled by the (even) ring period and its start aligned to it, so
// every register-ring index and the parity of every row are compile-time
// constants: no selects, static LDS offsets.
//
// Division by the diagonal 1-4*rr*nu uses the host-computed y = RN(1/d) and
// one Markstein correction: q0 = a*y, r = fma(-q0,d,a), q = fma(r,y,q0)
// (q0 if r == 0, which keeps the sign of a zero).  With y = RN(1/d) this is
// the correctly rounded quotient (Markstein's theorem), i.e. bitwise a/d;
// tools/check_division.c tests it on 1.4e9 random operands.
//
// MODE bits: 1 ZERO (u_in == 0, multigrid.cpp:77: no u loads); 2 PROLONG
// (u_in = uin + P(uc): the bilinear prolongation of the coarse correction,
// gs.cpp:238-265 expressions, added on load = multigrid.cpp:81-83 fused);
// 4 RESTRICT (residual at the fine even-even points written to the coarse
// rhs, multigrid.cpp:73-75 fused); 8 NORM (sum of squared residuals of the
// interior: per-workgroup partials, multigrid.cpp:112-113 fused).
//
// Work split (marches): a 1-D grid of workgroups, each with a share of the
// (strip, row) space (MarchRegions below), so one launch is one balanced wave.
struct RowData {
    double2 r, x, y;
};
// the four coefficients of a row's two points (column c0 in .x, c0+1 in .y):
// (rhs - cn*uN - cw*uW - cs*uS - ce*uE) / d, gs.cpp:126-130
struct CoefRow {
    double2 cn, cw, cs, ce;
};

// The sign of a/d is sign(a) xor sign(d), also for a = +-0 (where the fma
// chain alone would return +0 for a = -0): one v_xor + v_bfi on the high word
// instead of a compare and two selects.
//
// POSD (the diagonal d > 0, as for every nu <= 0): the same correction with
// the residual negated, rn = q0*d - a and q = fma(-rn, y, q0), is the same
// rounded value for every a != 0 (RN is symmetric) and gets the zero sign
// right by itself: a = -0 gives q0 = -0, rn = +0, q = -0 + -0 = -0; a = +0
// gives +0.  (For d < 0 it would not: a = +0 -> +0, not -0.)  Two integer ops
// fewer per point update; the launchers route d <= 0 to the general form.
template <bool POSD = false>
__device__ __forceinline__ double div_diag(double a, const Coef &c) {
    if (POSD) {
        const double q0 = a * c.rdgs;
        const double rn = __builtin_fma(q0, c.dgs, -a);
        return __builtin_fma(-rn, c.rdgs, q0);
    }
    const double q0 = a * c.rdgs;
    const double r = __builtin_fma(-q0, c.dgs, a);
    const double q = __builtin_fma(r, c.rdgs, q0);
    const long long qb = __double_as_longlong(q);
    const unsigned sh = (unsigned)(__double_as_longlong(a) >> 32) ^ c.dsign;
    const unsigned qh = ((unsigned)(qb >> 32) & 0x7fffffffu) | (sh & 0x80000000u);
    return __longlong_as_double(((long long)qh << 32) | (unsigned)qb);
}
// gs.cpp:130 with the Markstein division (bitwise equal to gs_point).
__device__ __forceinline__ double gs_point_fast(double rhs, double v1, double v2, double uN,
                                                double uW, double uS, double uE,
                                                const Coef &c) {
    const double aa = coef_a(v2, c), bb = coef_b(v2, c);
    const double cc = coef_a(v1, c), dd = coef_b(v1, c);
    return div_diag(rhs - cc * uN - aa * uW - dd * uS - bb * uE, c);
}

template <int K, int MODE>
struct SmoothCfg {
    static constexpr bool ZERO = (MODE & 1) != 0;
    static constexpr bool PROL = (MODE & 2) != 0;
    static constexpr bool REST = (MODE & 4) != 0;
    static constexpr bool NORM = (MODE & 8) != 0;
    static constexpr int S = 2 * K;                      // smoothing stages
    static constexpr int E = S + ((REST || NORM) ? 1 : 0);  // + residual stage
    static constexpr int H = (E + 1) / 2;                // halo pairs per side
    static constexpr int NR = E + 3;                     // LDS ring rows
    static constexpr int NS = S + 2;                     // register ring rows / unroll
};

// Work of one march launch (k_wsmooth, k_xsmooth): up to 4 rectangles of
// (strip group, row) units, enumerated group-major.  Region k covers strips
// [sfirst, slim) in groups of WPB (the waves / pairs of a workgroup; those of a
// last, partial group past slim idle) and rows [r0, r1); pre[] are the prefix
// unit counts (groups x rows).  band[k] > 0: the region is enumerated
// band-major instead -- bands of band[k] rows, group-major inside a band --
// so that with band[k] = units per workgroup, workgroup (band b, group j)
// marches rows [r0 + b*band, +band) of group j and the workgroups of
// neighbouring groups march the same rows at the same time.  xcd = 1: the
// workgroup order is dealt XCD-contiguous (wg_order).  seg = 1 (one region,
// band[0] > 0): workgroup (band b, group j) marches exactly that segment,
// also in a shorter last band (march_units): with units_per_wg = band the
// workgroups of a partial last band would each march pieces of several
// groups, each paying a warm-up.
struct MarchRegions {
    int sfirst[4], slim[4], r0[4], r1[4];
    int band[4];
    long pre[5];
    int count;
    int xcd;
    int seg;
};
// -> (strip of wave / pair `w` of the group, a, b) of the segment starting at
// unit `start` (at most `end`); strip < 0: this wave idles on the segment.
__device__ __forceinline__ void region_segment(const MarchRegions &reg, int wpb, int w,
                                               long start, long end, int &strip, int &a,
                                               int &b) {
    int k = 0;
    while (start >= reg.pre[k + 1]) ++k;
    long loc = start - reg.pre[k];
    int r0 = reg.r0[k], nr = reg.r1[k] - reg.r0[k];
    if (reg.band[k] > 0) {   // band-major: (band, group, row)
        const int ng = (reg.slim[k] - reg.sfirst[k] + wpb - 1) / wpb;
        const long per = (long)ng * reg.band[k];
        const int bi = (int)(loc / per);
        loc -= bi * per;
        r0 += bi * reg.band[k];
        nr = min(reg.band[k], nr - bi * reg.band[k]);
    }
    strip = reg.sfirst[k] + (int)(loc / nr) * wpb + w;
    if (strip >= reg.slim[k]) strip = -1;
    a = r0 + (int)(loc % nr);
    b = (int)min((long)(r0 + nr), (long)a + (end - start));
}

// Logical workgroup index of a march launch.  Workgroups are dealt
// round-robin over the 8 XCDs (b and b+8 share one, MI355X_MICROARCH
// "Workgroup dispatch"); reg.xcd = 1 gives each XCD a contiguous run of
// logical indices -- neighbouring strip groups of a band -- so the halo
// columns two neighbours both read are fetched once into that XCD's L2.
__device__ __forceinline__ long wg_order(const MarchRegions &reg) {
    const int b = blockIdx.x;
    if (!reg.xcd) return b;
    const int G = gridDim.x, q = G >> 3, r = G & 7, x = b & 7;
    return (long)x * q + min(x, r) + (b >> 3);
}

// The units [start, end) a workgroup of a march launch works on.
__device__ __forceinline__ void march_units(const MarchRegions &reg, int wpb, long upw,
                                            long &start, long &end) {
    const long w = wg_order(reg);
    if (!reg.seg) {
        start = w * upw;
        end = min(reg.pre[reg.count], start + upw);
        return;
    }
    const int ng = (reg.slim[0] - reg.sfirst[0] + wpb - 1) / wpb;
    const int B = reg.band[0], rows = reg.r1[0] - reg.r0[0];
    const int bb = (int)(w / ng), j = (int)(w % ng);
    const int h = max(0, min(B, rows - bb * B));
    start = (long)bb * ng * B + (long)j * h;
    end = start + h;
}

// k_wsmooth: the fused K-sweep pass (temporal blocking above) as a WAVE-PRIVATE march.
//
// One workgroup = one wave of 64 lanes; lane l owns the column pair
// (c0, c0+1), c0 = j0 - 2H + 2l.  Everything a stage needs lives in the
// wave's own registers: a ring of u rows (double2 per lane), the rhs / v1 /
// v2 ring (RowData per lane), and the west / east neighbour columns come
// from the adjacent lanes by DPP wave shifts (v_mov_b32_dpp wave_shr:1 /
// wave_shl:1).  No LDS and no barriers: the stage chain is a short run of
// dependent fp64 VALU ops, and the two to three waves per SIMD overlap.
//
// Schedule: at step s stage h (h = 0..S-1, S = 2K) updates
// its colour in row s+1-h; the residual stage (RESTRICT / NORM) takes row
// s+1-S; row s+2-S is final and stored.  u rows s-S .. s+3 are live (S+4 =
// NR rows), rhs/v rows s+1-S .. s+WRV (loaded WRV steps ahead, MGX_WRV);
// NR is even and the step loop is unrolled NR times with its start
// aligned to NR, so every ring index and every row parity is a compile-time
// constant.
//
// The exact cone, halo lanes (H = ceil(E/2) pairs per side), clamped
// unconditional loads, Markstein division and modes are those above;
// each exact value is computed from exactly the operands of the sequential
// gs.cpp sweeps (bitwise).  The velocity terms enter as t = v*(h/2), which
// is bitwise v*h/2.0 (scaling by 2^-1 is exact for these magnitudes), so a(v)
// = rr*(nu - t) and b(v) = rr*(t + nu) exactly as gs.cpp:14-20.
template <int K, int MODE>
struct WCfg {
    static constexpr bool ZERO = (MODE & 1) != 0;
    static constexpr bool PROL = (MODE & 2) != 0;
    static constexpr bool REST = (MODE & 4) != 0;
    static constexpr bool NORM = (MODE & 8) != 0;
    // RHSN: the rhs is computed on the fly from the (original) u rows as they
    // enter the ring (gs.cpp:44), stored, and the residual of u against it
    // summed (mg_outer's initial norm, multigrid.cpp:104) -- a time step's
    // compute_rhs, initial norm and first pre-smoothing in one pass
    static constexpr bool RHSN = (MODE & 16) != 0;
    static constexpr int S = 2 * K;
    static constexpr int E = S + ((REST || NORM) ? 1 : 0);
    static constexpr int H = (E + 1) / 2;
    static constexpr int NR = S + 4;   // u ring = rhs/v ring = unroll period (even)
    static constexpr int W = 2 * (64 - 2 * H);
    // rows an unguarded march may own: its warm-up updates rows down to
    // E + NR + S - 2 above the first, its drain E - 2 below the last
    static constexpr int TOP = E + NR + S + 2, BOT = E + 4;
};

// rhs/v prefetch distance of the wave march: with t = v*h/2 formed at the
// row's first use (scale_rv), 4 steps measured -3 % on level 1 against 2
// (3: -2 %, 5: -2 %; tools/ab_libs.sh)
#ifndef MGX_WRV
#define MGX_WRV 4
#endif

// 64-bit value of lane l-1 (shr) / l+1 (shl); the edge lane reads 0
// (bound_ctrl: one v_mov_b32_dpp per half, no zeroing move)
__device__ __forceinline__ double dpp_shr1(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x138, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double dpp_shl1(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x130, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// the same shifts, the edge lane (0 / 63) keeping `old` (bound_ctrl off:
// its write is disabled, so the v_mov_b32_dpp leaves the old value in place)
__device__ __forceinline__ double dpp_shr1_or(double v, double old) {
    const long long b = __double_as_longlong(v), o = __double_as_longlong(old);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), 0x138, 0xf, 0xf,
                                               false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double dpp_shl1_or(double v, double old) {
    const long long b = __double_as_longlong(v), o = __double_as_longlong(old);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), 0x130, 0xf, 0xf,
                                               false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// gs.cpp:130 / :75 with the velocity terms pre-scaled: t1 = v1*h/2, t2 = v2*h/2
template <bool POSD = false>
__device__ __forceinline__ double gs_point_t(double rhs, double t1, double t2, double uN,
                                             double uW, double uS, double uE, const Coef &c) {
    const double aa = c.rr * (c.nu - t2), bb = c.rr * (t2 + c.nu);
    const double cc = c.rr * (c.nu - t1), dd = c.rr * (t1 + c.nu);
    return div_diag<POSD>(rhs - cc * uN - aa * uW - dd * uS - bb * uE, c);
}
__device__ __forceinline__ double res_point_t(double rhs, double t1, double t2, double u,
                                              double uN, double uW, double uS, double uE,
                                              const Coef &c) {
    const double aa = c.rr * (c.nu - t2), bb = c.rr * (t2 + c.nu);
    const double cc = c.rr * (c.nu - t1), dd = c.rr * (t1 + c.nu);
    return rhs - (c.dgs * u + cc * uN + aa * uW + dd * uS + bb * uE);
}
// gs.cpp:44 with t1, t2
__device__ __forceinline__ double rhs_point_t(double t1, double t2, double u, double uN,
                                              double uW, double uS, double uE, const Coef &c) {
    const double aa = c.rr * (c.nu - t2), bb = c.rr * (t2 + c.nu);
    const double cc = c.rr * (c.nu - t1), dd = c.rr * (t1 + c.nu);
    return c.drhs * u - cc * uN - aa * uW - dd * uS - bb * uE;
}

// G = false: the unguarded march (interior strips, rows [TOP, n+1-BOT) of
// WCfg: no per-stage predicates), G = true: guarded (see k_xsmooth).
// PD: the diagonal is positive (every nu <= 0): the shorter division (div_diag).
// MGX_WCOEF: each row's four coefficients are formed once, at its first stage
// (as in k_xsmooth), instead of in every stage of its points.
// (2: only the x-neighbour pair cn, cs, from t1 -- half the registers of all
// four -- the y pair from t2 in every stage)
#ifndef MGX_WCOEF
#define MGX_WCOEF 2
#endif
template <int WPB, int K, int MODE, bool G, bool PD = false>
__global__ __launch_bounds__(64 * WPB) void k_wsmooth(
    const double *__restrict__ uin, double *__restrict__ uout, const double *__restrict__ rhs,
    const double *__restrict__ v1, const double *__restrict__ v2, const double *__restrict__ uc,
    long pitchc, double *__restrict__ rhsc, double *__restrict__ partials, int n, long pitch,
    MarchRegions reg, long units_per_wg, Coef c, int lo, int hi, double *__restrict__ rhs_out,
    const double *__restrict__ zrow, int vz) {
    using C = WCfg<K, MODE>;
    constexpr int S = C::S, E = C::E, H = C::H, NR = C::NR, W = C::W;
    // rhs/v prefetch distance in steps (row s+WRV takes the slot of row
    // s+WRV-NR, last used by the residual stage on row s+1-S); RHSN uses a
    // row's v two steps before its first stage
    constexpr int WRV = C::RHSN ? (MGX_WRV > 4 ? MGX_WRV : 4) : MGX_WRV;
    static_assert(WRV >= 2 && WRV <= NR - S + 1, "rhs/v prefetch distance");
    // WPB waves per workgroup march WPB adjacent strips over the same rows,
    // independently (no barriers); their row loads are adjacent 1-KiB pieces
    // of the same rows, issued at about the same time
    const int l = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    long start, end;
    march_units(reg, WPB, units_per_wg, start, end);
    const int nc = n >> 1;
    const double hh = c.h * 0.5;
    double acc = 0.0;
    // row offsets as 32 x 32 -> 64-bit products (pitches < 2^31 elements)
    const int ip = (int)pitch, ipc = (int)pitchc;
    auto rowoff = [](int r, int p) { return (long)r * (long)p; };
    int a = 0, b = 0;   // the segment's owned rows (set per segment below)
    // r in [a, b) as one unsigned compare (b >= a)
    auto rowin = [&](int r) { return (unsigned)(r - a) < (unsigned)(b - a); };

    while (start < end) {
        int strip;   // a, b: the segment's rows (captured by rowin)
        region_segment(reg, WPB, wv, start, end, strip, a, b);
        start += b - a;
        if (__builtin_amdgcn_readfirstlane(strip) < 0) continue;

        const int j0 = strip * W;
        const int c0 = j0 - 2 * H + 2 * l;
        const bool act = c0 >= 0 && c0 <= n;
        const bool keep = act && l >= H && l < 64 - H;
        const bool in0 = act && c0 >= 1 && c0 <= n - 1;
        const bool in1 = act && c0 + 1 <= n - 1;

        struct UPre {
            double2 X;
            double q00, q01, q10, q11;
        };
        UPre up[2];
        up[0] = up[1] = UPre{make_double2(0.0, 0.0), 0.0, 0.0, 0.0, 0.0};
        const int cl = min(max(c0, 0), (int)pitch - 2);
        const int jl = cl >> 1;
        const int j1 = (jl + 1 <= nc) ? 1 : 0;
        // (odd = R's parity, a compile-time constant at every call site: an
        // even row's prolongation needs only the coarse row below it)
        auto load_u = [&](int R, UPre &u, const bool odd) {
            if (C::ZERO) return;
            const int Rc = min(max(R, lo), hi);
            u.X = ld2((uin + rowoff(Rc, ip)) + cl);
            if (C::PROL) {
                const double *p0 = (uc + rowoff(Rc >> 1, ipc)) + jl;
                u.q00 = p0[0];
                u.q01 = p0[j1];
                if (odd) {
                    u.q10 = p0[ipc];
                    u.q11 = p0[ipc + j1];
                }
            }
        };
        // u row R (+ prolongation) as it enters the ring
        // (row parity `odd` is a compile-time constant at every call site; the
        // range test is a select: branches here make the waitcnt pass drain
        // the prefetch queue)
        auto make_u = [&](int R, const UPre &u, const bool odd) {
            double2 v = u.X;
            if (C::ZERO) v = make_double2(0.0, 0.0);
            if (C::PROL) {
                double2 pr;
                const double q01 = (!G || j1) ? u.q01 : 0.0;
                const double q11 = (!G || j1) ? u.q11 : 0.0;
                if (!odd) {
                    pr.x = u.q00;
                    pr.y = (u.q00 + q01) / 2;
                } else {
                    pr.x = (u.q00 + u.q10) / 2;
                    pr.y = (u.q00 + u.q10 + q01 + q11) / 4;
                }
                const bool on = !G || (act && R >= 0 && R <= n);
                v.x = on ? v.x + pr.x : v.x;
                v.y = on ? v.y + pr.y : v.y;
            }
            return v;
        };
        // rhs and v of row R, raw; t = v*h/2 only at the row's first use
        // (scale_rv): scaled here, the multiplies would wait for the loads
        // right after issuing them, and no prefetch distance would help
        // (rows >= vz: v1 and v2 are zero there, read from the L2-resident
        // zero row -- a uniform select, the load stays unconditional)
        auto load_rv = [&](int R, RowData &d) {
            const int Rc = min(max(R, lo), hi);
            const long o = rowoff(Rc, ip);
            if (!C::RHSN) d.r = ld2((rhs + o) + cl);
            const bool z = Rc >= vz;
            d.x = ld2((z ? zrow : v1 + o) + cl);
            d.y = ld2((z ? zrow : v2 + o) + cl);
        };
        auto scale_rv = [&](RowData &d) {
            d.x = make_double2(d.x.x * hh, d.x.y * hh);
            d.y = make_double2(d.y.x * hh, d.y.y * hh);
        };

        const int s_first = a - E;
        const int s_last = b + E - 3;
        int s = s_first >= 0 ? (s_first / NR) * NR : -(((-s_first) + NR - 1) / NR) * NR;
        s = __builtin_amdgcn_readfirstlane(s);

        double2 ur[NR];
        RowData rd[NR];
        constexpr bool WC = MGX_WCOEF == 1 && !C::RHSN;
        constexpr bool WH = MGX_WCOEF == 2 && !C::RHSN;   // half: cn, cs stored
        CoefRow cf[NR];
#pragma unroll
        for (int q = 0; q < NR; ++q) {
            ur[q] = make_double2(0.0, 0.0);
            rd[q].r = rd[q].x = rd[q].y = make_double2(0.0, 0.0);
            const double2 z = make_double2(0.0, 0.0);
            cf[q] = CoefRow{z, z, z, z};
        }
        // gs.cpp:126-129 coefficients of a row's two points from t1, t2
        auto to_coef = [&](const RowData &d, CoefRow &k) {
            k.cn = make_double2(c.rr * (c.nu - d.x.x), c.rr * (c.nu - d.x.y));
            k.cw = make_double2(c.rr * (c.nu - d.y.x), c.rr * (c.nu - d.y.y));
            k.cs = make_double2(c.rr * (d.x.x + c.nu), c.rr * (d.x.y + c.nu));
            k.ce = make_double2(c.rr * (d.y.x + c.nu), c.rr * (d.y.y + c.nu));
        };
        // residual (gs.cpp:75 term order) of the row in slot iR, column c0 / c0+1
        auto res_cx = [&](const int iR, const int iN, const int iS, const double uW) {
            const CoefRow &k = cf[iR];
            const double cw = MGX_WCOEF == 2 ? c.rr * (c.nu - rd[iR].y.x) : k.cw.x;
            const double ce = MGX_WCOEF == 2 ? c.rr * (rd[iR].y.x + c.nu) : k.ce.x;
            return rd[iR].r.x - (c.dgs * ur[iR].x + k.cn.x * ur[iN].x + cw * uW +
                                 k.cs.x * ur[iS].x + ce * ur[iR].y);
        };
        auto res_cy = [&](const int iR, const int iN, const int iS, const double uE) {
            const CoefRow &k = cf[iR];
            const double cw = MGX_WCOEF == 2 ? c.rr * (c.nu - rd[iR].y.y) : k.cw.y;
            const double ce = MGX_WCOEF == 2 ? c.rr * (rd[iR].y.y + c.nu) : k.ce.y;
            return rd[iR].r.y - (c.dgs * ur[iR].y + k.cn.y * ur[iN].y + cw * ur[iR].x +
                                 k.cs.y * ur[iS].y + ce * uE);
        };
        // prologue (s == 0 mod NR): u rows s..s+2 in the ring, s+3 / s+4 in
        // flight (sets 1 / 0), rhs/v rows s+1, s+2 loaded
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            load_u(s + d, up[0], d & 1);
            ur[d] = make_u(s + d, up[0], d & 1);
        }
        load_u(s + 3, up[1], true);
        load_u(s + 4, up[0], false);
#pragma unroll
        for (int d = 1; d < WRV; ++d) load_rv(s + d, rd[d]);
        // RHSN: rhs of row r (ring slot iR) from its original u rows r-1..r+1,
        // stored on the owned interior points, and the residual of u against
        // it summed (gs.cpp:44, :75; interior, owned rows / lanes only)
        auto rhs_norm = [&](const int r, const int iR, const int iN, const int iS) {
            RowData &d = rd[iR];
            const double uW = dpp_shr1(ur[iR].y), uE = dpp_shl1(ur[iR].x);
            // a fresh scalar nu: keeps the compiler from holding this row's
            // coefficients live until its smoothing stages (MGX_RHSN_CSE)
            Coef cg = c;
#ifndef MGX_RHSN_CSE
            asm volatile("" : "+s"(cg.nu));
#endif
            const double f0 = rhs_point_t(d.x.x, d.y.x, ur[iR].x, ur[iN].x, uW, ur[iS].x,
                                          ur[iR].y, cg);
            const double f1 = rhs_point_t(d.x.y, d.y.y, ur[iR].y, ur[iN].y, ur[iR].x, ur[iS].y,
                                          uE, cg);
            d.r = make_double2(f0, f1);
            if (rowin(r) && r >= 1 && r <= n - 1 && keep) {
                double *row = rhs_out + rowoff(r, ip);
                if (in0 && in1) {
                    st2(row + c0, d.r);
                } else {
                    if (in0) row[c0] = f0;
                    if (in1) row[c0 + 1] = f1;
                }
                if (in0) {
                    const double res = res_point_t(f0, d.x.x, d.y.x, ur[iR].x, ur[iN].x, uW,
                                                   ur[iS].x, ur[iR].y, c);
                    acc += res * res;
                }
                if (in1) {
                    const double res = res_point_t(f1, d.x.y, d.y.y, ur[iR].y, ur[iN].y,
                                                   ur[iR].x, ur[iS].y, uE, c);
                    acc += res * res;
                }
            }
        };
        if (C::RHSN) {
            scale_rv(rd[1]);
            rhs_norm(s + 1, 1, 0, 2);   // the first stage's row
        }

        for (;;) {
#pragma unroll
            for (int p = 0; p < NR; ++p) {
                // (1) u row s+3 enters the ring; its prefetch set takes row s+5
                ur[(p + 3) % NR] = make_u(s + 3, up[(p + 1) & 1], (p + 3) & 1);
                load_u(s + 5, up[(p + 1) & 1], (p + 1) & 1);
                // t of the row first used in this step: s+2 (RHSN), else s+1
                scale_rv(rd[(p + (C::RHSN ? 2 : 1)) % NR]);
                if (WC) to_coef(rd[(p + 1) % NR], cf[(p + 1) % NR]);
                if (WH) {   // cn, cs of row s+1 from t1 (gs.cpp:128-129's cc, dd)
                    const RowData &d1 = rd[(p + 1) % NR];
                    CoefRow &k1 = cf[(p + 1) % NR];
                    k1.cn = make_double2(c.rr * (c.nu - d1.x.x), c.rr * (c.nu - d1.x.y));
                    k1.cs = make_double2(c.rr * (d1.x.x + c.nu), c.rr * (d1.x.y + c.nu));
                }
                // rows s+1..s+3 are still original u: rhs of row s+2
                if (C::RHSN) rhs_norm(s + 2, (p + 2) % NR, (p + 1) % NR, (p + 3) % NR);
                // (2) the S smoothing stages
#pragma unroll
                for (int h = 0; h < S; ++h) {
                    const int r = s + 1 - h;
                    const int iR = (p + 1 - h + 2 * NR) % NR;
                    const int iN = (p - h + 2 * NR) % NR;
                    const int iS = (p + 2 - h + 2 * NR) % NR;
                    const int cs = ((p + 1 - h) & 1) ^ (h & 1);
                    const RowData &d = rd[iR];
                    // (one unsigned compare: r in [1, n-1])
                    const bool inr = !G || (unsigned)(r - 1) < (unsigned)(n - 1);
                    // unguarded: fresh scalar nu per stage (no cross-stage
                    // coefficient CSE: it would need more VGPRs, see k_xsmooth)
                    Coef cg = c;
                    if (!G) asm volatile("" : "+s"(cg.nu));
                    const CoefRow &k = cf[iR];
                    if (cs == 0) {
                        const double uW = dpp_shr1(ur[iR].y);   // column c0-1
                        if (!G || (inr && in0)) {
                            if (WH)
                                ur[iR].x = div_diag<PD>(d.r.x - k.cn.x * ur[iN].x -
                                                            cg.rr * (cg.nu - d.y.x) * uW -
                                                            k.cs.x * ur[iS].x -
                                                            cg.rr * (d.y.x + cg.nu) * ur[iR].y,
                                                        c);
                            else if (WC)
                                ur[iR].x = div_diag<PD>(d.r.x - k.cn.x * ur[iN].x - k.cw.x * uW -
                                                            k.cs.x * ur[iS].x - k.ce.x * ur[iR].y,
                                                        c);
                            else
                                ur[iR].x = gs_point_t<PD>(d.r.x, d.x.x, d.y.x, ur[iN].x, uW,
                                                          ur[iS].x, ur[iR].y, cg);
                        }
                    } else {
                        const double uE = dpp_shl1(ur[iR].x);   // column c0+2
                        if (!G || (inr && in1)) {
                            if (WH)
                                ur[iR].y = div_diag<PD>(d.r.y - k.cn.y * ur[iN].y -
                                                            cg.rr * (cg.nu - d.y.y) * ur[iR].x -
                                                            k.cs.y * ur[iS].y -
                                                            cg.rr * (d.y.y + cg.nu) * uE,
                                                        c);
                            else if (WC)
                                ur[iR].y = div_diag<PD>(d.r.y - k.cn.y * ur[iN].y -
                                                            k.cw.y * ur[iR].x - k.cs.y * ur[iS].y -
                                                            k.ce.y * uE,
                                                        c);
                            else
                                ur[iR].y = gs_point_t<PD>(d.r.y, d.x.y, d.y.y, ur[iN].y, ur[iR].x,
                                                          ur[iS].y, uE, cg);
                        }
                    }
                }
                // (3) row s+2-S is final
                {
                    const int ro = s + 2 - S;
                    st2_if(uout + rowoff(ro, ip), c0, rowin(ro) && keep,
                           ur[(p + 2 - S + 2 * NR) % NR]);
                }
                // (4) residual stage on row s+1-S
                if (C::REST || C::NORM) {
                    const int r = s + 1 - S;
                    const int iR = (p + 1 - S + 2 * NR) % NR;
                    const int iN = (p - S + 2 * NR) % NR;
                    const int iS = (p + 2 - S + 2 * NR) % NR;
                    const RowData &d = rd[iR];
                    const double uW = dpp_shr1(ur[iR].y);
                    // (the same expressions from the row's coefficients, bitwise)
                    auto rx = [&]() {
                        if (WC || WH) return res_cx(iR, iN, iS, uW);
                        return res_point_t(d.r.x, d.x.x, d.y.x, ur[iR].x, ur[iN].x, uW, ur[iS].x,
                                           ur[iR].y, c);
                    };
                    if (C::REST) {
                        if (((p + 1 - S) & 1) == 0 && rowin(r) && keep &&
                            (!G || (r >= 1 && r <= n - 2 && in0 && c0 <= n - 2))) {
                            const double res = rx();
                            (rhsc + rowoff(r >> 1, ipc))[c0 >> 1] = res;
                        }
                    } else {
                        const double uE = dpp_shl1(ur[iR].x);
                        auto ry = [&]() {
                            if (WC || WH) return res_cy(iR, iN, iS, uE);
                            return res_point_t(d.r.y, d.x.y, d.y.y, ur[iR].y, ur[iN].y, ur[iR].x,
                                               ur[iS].y, uE, c);
                        };
                        if (!G) {   // acc + 0.0 == acc (acc >= +0): selects, no branch
                            if (rowin(r)) {
                                const double r0 = rx();
                                const double r1 = ry();
                                acc += keep ? r0 * r0 : 0.0;
                                acc += keep ? r1 * r1 : 0.0;
                            }
                        } else if (keep && rowin(r) && r >= 1 && r <= n - 1) {
                            if (in0) {
                                const double res = rx();
                                acc += res * res;
                            }
                            if (in1) {
                                const double res = ry();
                                acc += res * res;
                            }
                        }
                    }
                }
                // (5) rhs/v row s+WRV into the slot of row s+WRV-NR (dead)
                load_rv(s + WRV, rd[(p + WRV) % NR]);
                if (++s > s_last) goto done;
            }
        }
    done:;
    }
    if (C::NORM || C::RHSN) {
        const double tot = wave_sum(acc);
        if (l == 0) partials[(long)blockIdx.x * WPB + wv] = tot;
    }
}

// k_xsmooth: the finest level's post-smoothing of V-cycle k FUSED with the
// pre-smoothing of V-cycle k+1 (software pipelining across cycles): in
// mg_outer the two are consecutive sweeps of level 0 with only the residual
// norm between them (multigrid.cpp:83-88 of cycle k, :112-113, :69-75 of
// cycle k+1), so one HBM pass can do both, reading rhs / v1 / v2 / u once.
//
// Workgroup = WPB pairs of waves on WPB adjacent strips.  In each pair, wave
// A runs the k_wsmooth march of the post-smoothing (prolongation + add on
// load, K sweeps, residual-norm partials) and wave B, D = S+4 rows behind,
// the march of the next pre-smoothing (K sweeps, residual restricted to the
// coarse rhs).  A hands B each finished u row and each rhs / v row through a
// small LDS ring (one lane to the same lane: no bank conflicts).  The march
// advances in PAIRS of steps: one barrier and one exit test per pair keep the
// waves D rows apart (B reads only rows A wrote in an earlier pair; half the
// barriers of a per-step hand-off: -2.5 % on the pass).  Register footprint
// per wave = that of one K-sweep march.  A also stores u_post (the solution after cycle k,
// which mg_outer returns if cycle k converged); B stores u_pre (cycle k+1
// after its pre-smoothing).  Exactness: B's output strip needs A's output
// on a cone EB = S+1 wider, A's on S more: H = ceil((S+EB)/2) halo pairs.
#ifndef MGX_XRV
#define MGX_XRV 4
#endif
#ifndef MGX_XU
#define MGX_XU 2
#endif
#ifndef MGX_XACOEF
#define MGX_XACOEF 1
#endif
// fewest rows per workgroup of the guarded edge launch
#ifndef MGX_XEDGE_ROWS
#define MGX_XEDGE_ROWS 16
#endif
template <int K>
struct XCfg {
    static constexpr int S = 2 * K;
    static constexpr int EB = S + 1;             // B: stages + restriction residual
    static constexpr int EA = S + 1;             // A: stages + norm residual
    static constexpr int H = (S + EB + 1) / 2;   // halo pairs per side
    static constexpr int NR = S + 4;             // register rings / unroll period
    static constexpr int W = 2 * (64 - 2 * H);
    static constexpr int D = S + 4;              // B's lag in rows
    // LDS hand-off rings, sizes dividing NR so every slot index is static.
    // Per pair of steps A writes u rows s+2-S, s+3-S and rhs/v rows s+1, s+2;
    // B reads u rows s-S-1, s-S and rhs/v rows s-S-1, s-S: spans of 5 and
    // S+4 = NR rows, no slot written and read in the same pair.
    static constexpr int NU = (NR % 5 == 0) ? 5 : NR, NRD = NR;
    // Rows an unguarded march may own: its warm-up reaches EA + EB + NR + D +
    // S rows above its first owned row and its drain D + EB + NR + 5 below its
    // last (B's garbage-in warm-up steps included), all of which must be rows
    // in [1, n-1] so that no update ever lands on a Dirichlet row.
    // (+1: the march runs an even number of steps)
    static constexpr int TOP = EA + EB + NR + D + S + 2, BOT = D + EB + NR + 7;
    // step mode (RS): B's march has one more stage in front (the next time
    // step's rhs from u_post), so A starts one row earlier: 2 more margin rows
    // (even) for the unguarded form; the halo H is unchanged (S + EB + 1 =
    // 14 columns fit its 7 pairs)
    static constexpr int TOP_RS = TOP + 2;
};


//
// G = true: the guarded march (rows / columns may touch the Dirichlet
// boundary; every stage tests them).  G = false: the unguarded march for
// interior strips (every lane a column in [1, n-1]) on rows [TOP, n+1-BOT),
// whose warm-up and drain stay in rows [1, n-1]: no per-stage predicates, so
// no exec-mask branches, -26 % instructions.  They are separate kernels: one
// function holding both marches compiled to a worse schedule than either
// (3.6 ms vs 2.7 ms unguarded / 3.1 ms guarded at N=16384).
//
// RS = true (time-step mode, mg_outer's last cycle of a time step whose next
// step follows): B's pre-smoothing is the NEXT time step's first one.  B
// forms the next step's rhs of each row from the final u_post rows as they
// arrive (gs.cpp:44, the expressions of rhs_point_t), stores it to rhs_next,
// sums the residual of u_post against it (the next mg_outer's initial norm,
// multigrid.cpp:104) into partials2, and smooths and restricts with it --
// the rhs + norm pass of the next step and this step's post-smoothing pass
// in one HBM pass.  (B's half of the u_post norm still uses this step's rhs.)
//
// SV = true (separable velocity, sepvel.h): v1[R][c] = fl(sa1[R] * sb1[c]) and
// v2 likewise, exactly.  A then reads only rhs and u from HBM: per row it
// loads the two row factors with scalar loads into an SGPR ring (XRV steps
// ahead, like the rhs row) and forms t = v*h/2 at the row's first stage as
// fl(sa[R] * fl(sb[c]*h/2)) -- bitwise fl(v*h/2), the scalings by h/2 being
// exact (sepvel.h checks the range) -- from the lane's column factors, held
// in registers for the whole march.
//
// XG = true (group exchange, unguarded only): the WPB pairs of a workgroup
// march WPB ADJACENT 128-column strips that overlap by nothing, and the
// workgroup as a whole is one 64*WPB-lane strip with the H-pair halo only on
// its two outer sides: group g owns WGc = 128*WPB - 4H columns (484 instead of
// 4 x 100).  The columns a wave's edge lanes need from the neighbouring wave
// of the same role (lane 0 the west wave's column c0-1, lane 63 the east
// wave's column c0+2) come through LDS: all inputs of a march step's stages
// and residuals from a neighbouring column are results of the PREVIOUS step
// (a stage on row r updates one colour; the other colour of row r was last
// updated by the stage before, one step earlier, or is the row's initial
// value), so each wave posts, at the end of a step, lane 0's .x and lane 63's
// .y of every row it changed (and of the row that entered its ring), and a
// barrier per step (instead of per two steps) orders post and use.  The
// edge lane takes the posted value through the DPP shift's "keep old" form
// (bound_ctrl off): no extra VALU instruction.  The halo work of the pass
// drops from 28 of 128 columns to 28 of 512.
// rhs row prefetch distance of the XG kernel (its exchange values take the
// registers of one prefetched row)
#ifndef MGX_XGRV
#define MGX_XGRV 3
#endif
#ifndef MGX_XG_DBG
#define MGX_XG_DBG 0
#endif
struct XGeo {
    int x0, xl, xend, glast;   // XG: owned origin of group 0, origin of the last group, end
    int ec0, ec1, er0, er1;    // guarded kernel: [ec0, ec1) x [er0, er1) owned by the XG launch
};

template <int WPB, int K, bool G, bool RS = false, bool SV = false, bool XG = false>
__global__ __launch_bounds__(128 * WPB) void k_xsmooth(
    const double *__restrict__ uin, double *__restrict__ upost, double *__restrict__ upre,
    const double *__restrict__ rhs, const double *__restrict__ v1, const double *__restrict__ v2,
    const double *__restrict__ uc, long pitchc, double *__restrict__ rhsc,
    double *__restrict__ partials, int n, long pitch, MarchRegions reg, long units_per_wg, Coef c,
    int lo, int hi, int store_post, double *__restrict__ rhs_next,
    double *__restrict__ partials2, const double *__restrict__ sa1,
    const double *__restrict__ sb1, const double *__restrict__ sa2,
    const double *__restrict__ sb2, XGeo xg) {
    using X = XCfg<K>;
    constexpr int S = X::S, H = X::H, NR = X::NR, W = X::W, D = X::D, NU = X::NU,
                  NRD = X::NRD, EA = X::EA, EB = X::EB;
    static_assert(!XG || !G, "the group exchange is the unguarded kernel's");
    constexpr int WGc = 128 * WPB - 4 * H;
    // A's prefetch distances in steps: rhs/v rows XRV ahead of their first
    // stage, u rows (+ coarse parents) XU ahead of entering the ring.  The
    // pass is bound by loads in flight, not by VALU: rhs/v 2 -> 3 -> 4 steps
    // took level 0 -4 % and -3 % at the same VGPR count (B's path sets it);
    // u 3-4 steps or rhs/v 5 measured no better (N=16384, tools/ab_libs.sh).
    constexpr int XRV = XG ? MGX_XGRV : MGX_XRV;
    constexpr int XU = MGX_XU;
    // A forms each row's coefficients once (MGX_XACOEF; B always does).  Not
    // in the guarded edge kernel: there it takes the kernel past 256 VGPRs
    // (one wave per SIMD), and the edge launch is latency bound
    constexpr bool XACOEF = MGX_XACOEF != 0 && !G;
    static_assert(XU >= 1 && XU <= NR - 3, "u prefetch distance");
    // row s+XRV takes the ring slot of row s+XRV-NR, last used by A's norm of
    // row s+1-S
    static_assert(XRV >= 2 && XRV <= NR - S + 1, "rhs/v prefetch distance");
    __shared__ double2 uring[WPB][NU][64];
    // rhs / t1 / t2 planes: each hand-off access is 16 B per lane, unit stride
    __shared__ double2 rdring[WPB][NRD][3][64];
    // XG: per role and wave, lane 0's .x (xchx) and lane 63's .y (xchy) of
    // each ring row, slot = row mod NR (the register rings' index)
    // (entries 0 and WPB+1 of each role: the outer waves' outer neighbours,
    // never written -- read only by halo lanes -- so that a wave's own, west
    // and east entries sit at fixed offsets from one address)
    // [role][wave + 1][0: lane 0's .x, 1: lane 63's .y][slot]
    __shared__ double xch[XG ? 2 : 1][XG ? WPB + 2 : 1][2][XG ? NR : 1];

    const int l = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const bool isA = wv < WPB;   // wave-uniform role
    const int pr = isA ? wv : wv - WPB;
    long start, end;
    march_units(reg, WPB, units_per_wg, start, end);
    const int nc = n >> 1;
    const double hh = c.h * 0.5;
    double acc = 0.0, acc2 = 0.0;
    // row offsets as 32 x 32 -> 64-bit products (the pitches are < 2^31
    // elements): two scalar multiplies per row address instead of a 64-bit one
    const int ip = (int)pitch, ipc = (int)pitchc;
    auto rowoff = [](int r, int p) { return (long)r * (long)p; };

    // One march of the pair over owned rows [a, b) of the strip whose lane 0
    // is column cb, owning columns [k0, k1) (G: see above; the unguarded form
    // keeps only the uniform owned-row tests of its outputs)
    auto march = [&](const int cb, const int k0, const int k1, const int a, const int b) {
        constexpr bool GM = G, GS = G, GN = G;   // make_u / stage / residual guards
        const int c0 = cb + 2 * l;
        const bool act = c0 >= 0 && c0 <= n;
        // the guarded kernel beside an XG launch: rows [er0, er1) of columns
        // [ec0, ec1) are that launch's (one owner per output)
        const bool exc = G && c0 >= xg.ec0 && c0 < xg.ec1;
        const bool keep = act && c0 >= k0 && c0 < k1;
        // (rows [a, b) as one unsigned compare: b >= a)
        auto own = [&](const int r) {
            return (unsigned)(r - a) < (unsigned)(b - a) && keep &&
                   !(exc && r >= xg.er0 && r < xg.er1);
        };
        // XG: the neighbouring waves of this role (the outer waves' outer
        // edge lanes are halo: any value will do, their own slot)
        const int rl = isA ? 0 : 1;
        const int pw = pr, pme = pr + 1, pe = pr + 2;
        // west neighbour of column c0 / east neighbour of column c0+1 of the
        // row in ring slot i: DPP shifts, the edge lane's from the neighbouring
        // wave's post (XG) or 0 (a halo lane)
        auto nbw = [&](const double y, const int i) {
            if (!XG || MGX_XG_DBG == 1) return dpp_shr1(y);
            return dpp_shr1_or(y, xch[rl][pw][1][i]);
        };
        auto nbe = [&](const double x, const int i) {
            if (!XG || MGX_XG_DBG == 1) return dpp_shl1(x);
            return dpp_shl1_or(x, xch[rl][pe][0][i]);
        };
        // XG: at the end of a step at ring phase q, post lane 0's .x / lane
        // 63's .y of the rows its stages changed (stage h, row slot q+1-h,
        // updates .x iff its colour cs = 0) and of the row that entered the
        // ring (slot q+3)
        auto post_edges = [&](const double2 *ur, const int q) {
            if (!XG || MGX_XG_DBG == 2) return;
            if (l == 0) {
#pragma unroll
                for (int h = 0; h < S; ++h)
                    if ((((q + 1 - h) & 1) ^ (h & 1)) == 0)
                        xch[rl][pme][0][(q + 1 - h + 2 * NR) % NR] = ur[(q + 1 - h + 2 * NR) % NR].x;
                xch[rl][pme][0][(q + 3) % NR] = ur[(q + 3) % NR].x;
            }
            if (l == 63) {
#pragma unroll
                for (int h = 0; h < S; ++h)
                    if ((((q + 1 - h) & 1) ^ (h & 1)) == 1)
                        xch[rl][pme][1][(q + 1 - h + 2 * NR) % NR] = ur[(q + 1 - h + 2 * NR) % NR].y;
                xch[rl][pme][1][(q + 3) % NR] = ur[(q + 3) % NR].y;
            }
        };
        const bool in0 = act && c0 >= 1 && c0 <= n - 1;
        const bool in1 = act && c0 + 1 <= n - 1;
        const int cl = min(max(c0, 0), (int)pitch - 2);
        const int jl = cl >> 1;
        const int j1 = (jl + 1 <= nc) ? 1 : 0;
        // per-lane byte offsets of the loads (uniform row bases: saddr form)
        const unsigned bcl = (unsigned)cl * 8u, bjl = (unsigned)jl * 8u,
                       bjl1 = (unsigned)(jl + j1) * 8u;

        struct UPre {
            double2 X;
            double q00, q01, q10, q11;
        };
        RowData rd[NR];   // rhs / t1 / t2 rows (ring by row)
        // u rows + coarse parents in flight, a ring by row like rd
        UPre up[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) up[i] = UPre{make_double2(0.0, 0.0), 0.0, 0.0, 0.0, 0.0};
        // A: u row R + its coarse parents (odd = R's parity, compile-time:
        // an even row needs only the coarse row below it)
        auto load_u = [&](int R, UPre &u, const bool odd) {
            const int Rc = min(max(R, lo), hi);
            u.X = ld2u(uin + rowoff(Rc, ip), bcl);
            const double *p0 = uc + rowoff(Rc >> 1, ipc);
            u.q00 = ld1u(p0, bjl);
            u.q01 = ld1u(p0, bjl1);
            if (odd) {
                u.q10 = ld1u(p0 + ipc, bjl);
                u.q11 = ld1u(p0 + ipc, bjl1);
            }
        };
        // + prolongation (gs.cpp:238-265); static parity, select (see k_wsmooth)
        auto make_u = [&](int R, const UPre &u, const bool odd) {
            double2 v = u.X;
            double2 pv;
            const double q01 = (!GM || j1) ? u.q01 : 0.0;
            const double q11 = (!GM || j1) ? u.q11 : 0.0;
            if (!odd) {
                pv.x = u.q00;
                pv.y = (u.q00 + q01) / 2;
            } else {
                pv.x = (u.q00 + u.q10) / 2;
                pv.y = (u.q00 + u.q10 + q01 + q11) / 4;
            }
            const bool on = !GM || (act && R >= 0 && R <= n);
            v.x = on ? v.x + pv.x : v.x;
            v.y = on ? v.y + pv.y : v.y;
            return v;
        };
        // SV: the lane's column factors scaled by h/2 (exact), and a ring of
        // row factors (wave-uniform: SGPRs), slot q = the rd slot of the row
        double2 bh1 = make_double2(0.0, 0.0), bh2 = bh1;
        double ar1[NR], ar2[NR];
        if (SV) {
            const double2 b1 = ld2(sb1 + cl), b2 = ld2(sb2 + cl);
            bh1 = make_double2(b1.x * hh, b1.y * hh);
            bh2 = make_double2(b2.x * hh, b2.y * hh);
#pragma unroll
            for (int i = 0; i < NR; ++i) ar1[i] = ar2[i] = 0.0;
        }
        auto load_rv = [&](int R, const int q) {
            const int Rc = min(max(R, lo), hi);
            const long o = rowoff(Rc, ip);
            RowData &d = rd[q];
            d.r = ld2u(rhs + o, bcl);
            if (SV) {   // (32-bit byte offsets: the scalar loads' SGPR-offset form)
                ar1[q] = *reinterpret_cast<const double *>(rowb(sa1, (unsigned)Rc * 8u));
                ar2[q] = *reinterpret_cast<const double *>(rowb(sa2, (unsigned)Rc * 8u));
            } else {
                const double2 x = ld2((v1 + o) + cl), y = ld2((v2 + o) + cl);
                d.x = make_double2(x.x * hh, x.y * hh);
                d.y = make_double2(y.x * hh, y.y * hh);
            }
        };
        // SV: t of the row in slot q, at its first stage
        auto make_t = [&](const int q) {
            if (!SV) return;
            rd[q].x = make_double2(ar1[q] * bh1.x, ar1[q] * bh1.y);
            rd[q].y = make_double2(ar2[q] * bh2.x, ar2[q] * bh2.y);
        };
        // one red-black stage h of the march step at row phase p on row r
        auto stage = [&](double2 *ur, RowData *rd, const int p, const int h, const int r) {
            const int iR = (p + 1 - h + 2 * NR) % NR;
            const int iN = (p - h + 2 * NR) % NR;
            const int iS = (p + 2 - h + 2 * NR) % NR;
            const int cs = ((p + 1 - h) & 1) ^ (h & 1);
            const RowData &d = rd[iR];
            const bool inr = !GS || (r >= 1 && r <= n - 1);
            // unguarded: a fresh (scalar) copy of nu per stage, so the compiler
            // does not keep each point's four coefficients live across its three
            // stages (that CSE needs ~50 more VGPRs than the 256 of two waves
            // per SIMD: spills); guarded stages are branches, never CSE'd
            Coef cg = c;
            if (!GS) asm volatile("" : "+s"(cg.nu));
            // (the unguarded kernel only runs with d > 0: xsmooth_inst)
            if (cs == 0) {
                const double uW = nbw(ur[iR].y, iR);
                if (!GS || (inr && in0))
                    ur[iR].x = gs_point_t<!GS>(d.r.x, d.x.x, d.y.x, ur[iN].x, uW, ur[iS].x,
                                               ur[iR].y, cg);
            } else {
                const double uE = nbe(ur[iR].x, iR);
                if (!GS || (inr && in1))
                    ur[iR].y = gs_point_t<!GS>(d.r.y, d.x.y, d.y.y, ur[iN].y, ur[iR].x,
                                               ur[iS].y, uE, cg);
            }
        };

        // A's first step (aligned to NR so ring indices and parities are
        // static); B runs D steps behind; the last iteration is B's last step
        // (rounded up to whole pairs: an extra step stores nothing)
        // (XG: 2 rows earlier -- the prologue's first rows s0+1, s0+2 enter
        // the ring unposted, so the neighbouring waves' warm-up garbage
        // reaches 2 rows further down than a lone strip's)
        int s0 = a - EB - EA - (RS ? 1 : 0) - (XG ? 2 : 0);
        s0 = s0 >= 0 ? (s0 / NR) * NR : -(((-s0) + NR - 1) / NR) * NR;
        s0 = __builtin_amdgcn_readfirstlane(s0);
        const int iters = ((b + EB - 3) + D - s0 + 1 + 1) & ~1;
        const bool post = store_post != 0;

        double2 ur[NR];
#pragma unroll
        for (int q = 0; q < NR; ++q) {
            ur[q] = make_double2(0.0, 0.0);
            rd[q].r = rd[q].x = rd[q].y = make_double2(0.0, 0.0);
        }
        // B turns each rhs/v row's t1, t2 into the four coefficients of its
        // two points once (gs.cpp:126-129, the expressions of gs_point_t),
        // just before the row's first stage, instead of in each of the
        // point's three stages and its restriction residual: -12 % VALU per
        // pass, -3 % time (the same in A as well: -23 % VALU, no further
        // time, 254 instead of 224 VGPRs -- the pass is not issue bound)
        CoefRow cf[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const double2 z = make_double2(0.0, 0.0);
            cf[i] = CoefRow{z, z, z, z};
        }
        auto to_coef = [&](const RowData &d, CoefRow &k) {
            k.cn = make_double2(c.rr * (c.nu - d.x.x), c.rr * (c.nu - d.x.y));
            k.cw = make_double2(c.rr * (c.nu - d.y.x), c.rr * (c.nu - d.y.y));
            k.cs = make_double2(c.rr * (d.x.x + c.nu), c.rr * (d.x.y + c.nu));
            k.ce = make_double2(c.rr * (d.y.x + c.nu), c.rr * (d.y.y + c.nu));
        };
        // stage h at ring phase q on row r (as `stage`), from the coefficients
        auto stage_c = [&](const int q, const int h, const int r) {
            const int iR = (q + 1 - h + 2 * NR) % NR;
            const int iN = (q - h + 2 * NR) % NR;
            const int iS = (q + 2 - h + 2 * NR) % NR;
            const int cs = ((q + 1 - h) & 1) ^ (h & 1);
            const CoefRow &k = cf[iR];
            const double2 f = rd[iR].r;
            const bool inr = !GS || (r >= 1 && r <= n - 1);
            if (cs == 0) {
                const double uW = nbw(ur[iR].y, iR);
                if (!GS || (inr && in0))
                    ur[iR].x = div_diag<!GS>(f.x - k.cn.x * ur[iN].x - k.cw.x * uW -
                                                 k.cs.x * ur[iS].x - k.ce.x * ur[iR].y,
                                             c);
            } else {
                const double uE = nbe(ur[iR].x, iR);
                if (!GS || (inr && in1))
                    ur[iR].y = div_diag<!GS>(f.y - k.cn.y * ur[iN].y - k.cw.y * ur[iR].x -
                                                 k.cs.y * ur[iS].y - k.ce.y * uE,
                                             c);
            }
        };
        // residual (gs.cpp:75 term order) at column c0 of the row in slot iR
        auto res_x = [&](const int iR, const int iN, const int iS, const double uW) {
            const CoefRow &k = cf[iR];
            return rd[iR].r.x - (c.dgs * ur[iR].x + k.cn.x * ur[iN].x + k.cw.x * uW +
                                 k.cs.x * ur[iS].x + k.ce.x * ur[iR].y);
        };
        // one loop per role (a role branch inside the step would make the
        // waitcnt pass see A's pending loads on B's path and drain them)
        int it = 0;
        if (isA) {
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                load_u(s0 + d, up[d], d & 1);
                ur[d] = make_u(s0 + d, up[d], d & 1);
            }
#pragma unroll
            for (int d = 3; d < 3 + XU; ++d) load_u(s0 + d, up[d], d & 1);
#pragma unroll
            for (int d = 1; d < XRV; ++d) load_rv(s0 + d, d);
            for (;;) {
#pragma unroll
                for (int p = 0; p < NR; ++p) {   // s == p (mod NR)
                    const int s = s0 + it + (p & 1);
                    ur[(p + 3) % NR] = make_u(s + 3, up[(p + 3) % NR], (p + 3) & 1);
                    load_u(s + 3 + XU, up[(p + 3 + XU) % NR], (p + 3 + XU) & 1);   // XU ahead
                    make_t((p + 1) % NR);   // row s+1: first used by stage 0 below
                    if (XACOEF) {
                        // the row's four coefficients once (as B does), not in
                        // each of its point's stages
                        to_coef(rd[(p + 1) % NR], cf[(p + 1) % NR]);
#pragma unroll
                        for (int h = 0; h < S; ++h) stage_c(p, h, s + 1 - h);
                    } else {
#pragma unroll
                        for (int h = 0; h < S; ++h) stage(ur, rd, p, h, s + 1 - h);
                    }
                    // hand-off: rhs/v row s+1 (first used above), final u row s+2-S
                    {
                        const RowData &dh = rd[(p + 1) % NR];
                        double2(*slot)[64] = rdring[pr][(p + 1) % NRD];
                        slot[0][l] = dh.r;
                        slot[1][l] = dh.x;
                        slot[2][l] = dh.y;
                    }
                    {
                        const int ro = s + 2 - S;
                        const double2 uf = ur[(p + 2 - S + 2 * NR) % NR];
                        uring[pr][(p + 2 - S + 2 * NR) % NU][l] = uf;
                        st2_ifu(upost + rowoff(ro, ip), c0, post && own(ro),
                               uf);
                    }
                    // residual norm of u_post (multigrid.cpp:112-113), column c0 of
                    // row s+1-S (its neighbours are final now; B takes column c0+1:
                    // half each balances the pair's VALU work)
                    {
                        const int r = s + 1 - S;
                        const int iR = (p + 1 - S + 2 * NR) % NR;
                        const int iN = (p - S + 2 * NR) % NR;
                        const int iS = (p + 2 - S + 2 * NR) % NR;
                        const RowData &d = rd[iR];
                        const double uW = nbw(ur[iR].y, iR);
                        // (with the row's coefficients: the same expressions, bitwise)
                        // XG: the row's rhs / t1 / t2 from the hand-off ring
                        // (B takes them two steps later) and the coefficients
                        // formed here -- 8 fp64 ops more, but A keeps neither
                        // the row's coefficients nor its rhs for this step: 20
                        // VGPRs fewer on A's path, which sets the kernel's count
                        auto res0 = [&]() {
                            if (XG) {
                                double2(*slot)[64] = rdring[pr][(p + 1 - S + 2 * NRD) % NRD];
                                const double2 fr = slot[0][l], f1 = slot[1][l], f2 = slot[2][l];
                                return res_point_t(fr.x, f1.x, f2.x, ur[iR].x, ur[iN].x, uW,
                                                   ur[iS].x, ur[iR].y, c);
                            }
                            if (XACOEF) return res_x(iR, iN, iS, uW);
                            return res_point_t(d.r.x, d.x.x, d.y.x, ur[iR].x, ur[iN].x, uW,
                                               ur[iS].x, ur[iR].y, c);
                        };
                        if (GN) {
                            if (own(r) && r >= 1 && r <= n - 1 && in0) {
                                const double res = res0();
                                acc += res * res;
                            }
                        } else {   // acc + 0.0 == acc (acc >= +0): a select, no branch
                            const double r0 = res0();
                            acc += own(r) ? r0 * r0 : 0.0;
                        }
                    }
                    load_rv(s + XRV, (p + XRV) % NR);
                    post_edges(ur, p);
                    if (XG || (p & 1)) __syncthreads();
                    if (p & 1) {   // end of a pair (compile-time)
                        it += 2;
                        if (it >= iters) goto done_a;
                    }
                }
            }
        done_a:;
        } else {
            for (;;) {
#pragma unroll
                for (int p = 0; p < NR; ++p) {
                    const int s = s0 + it + (p & 1) - D;   // B's ring phase q = p - D (mod NR)
                    constexpr int dq = ((D % NR) + NR) % NR;
                    const int q = (p - dq + NR) % NR;   // compile-time after unrolling
                    // u row s+3 (A finished it in an earlier pair) and rhs/v row s+3
                    ur[(q + 3) % NR] = uring[pr][(q + 3) % NU][l];
                    {
                        double2(*slot)[64] = rdring[pr][(q + 3) % NRD];
                        rd[(q + 3) % NR].r = slot[0][l];
                        rd[(q + 3) % NR].x = slot[1][l];
                        rd[(q + 3) % NR].y = slot[2][l];
                    }
                    // residual norm of u_post (multigrid.cpp:112-113) on row s+2,
                    // column c0+1 (A takes c0): rows s+1..s+3 are still untouched
                    // u_post here
                    {
                        const int r = s + 2;
                        const int iR = (q + 2) % NR, iN = (q + 1) % NR, iS = (q + 3) % NR;
                        const RowData &d = rd[iR];
                        const double uE = nbe(ur[iR].x, iR);
                        if (GN) {
                            if (own(r) && r >= 1 && r <= n - 1 && in1) {
                                const double res =
                                    res_point_t(d.r.y, d.x.y, d.y.y, ur[iR].y, ur[iN].y,
                                                ur[iR].x, ur[iS].y, uE, c);
                                acc += res * res;
                            }
                        } else {   // acc + 0.0 == acc (acc >= +0): a select, no branch
                            const double r1 = res_point_t(d.r.y, d.x.y, d.y.y, ur[iR].y,
                                                          ur[iN].y, ur[iR].x, ur[iS].y, uE, c);
                            acc += own(r) ? r1 * r1 : 0.0;
                        }
                    }
                    if (RS) {
                        // the next step's rhs of row s+2 from u_post rows s+1..s+3
                        // (gs.cpp:44), stored on the owned interior points, and the
                        // residual of u_post against it (multigrid.cpp:104); it
                        // replaces this step's rhs in the ring for B's stages and
                        // restriction
                        const int r = s + 2;
                        const int iR = (q + 2) % NR, iN = (q + 1) % NR, iS = (q + 3) % NR;
                        RowData &d = rd[iR];
                        const double uW = nbw(ur[iR].y, iR), uE = nbe(ur[iR].x, iR);
                        Coef cg = c;   // fresh nu: no coefficient CSE into the stages
                        asm volatile("" : "+s"(cg.nu));
                        const double f0 = rhs_point_t(d.x.x, d.y.x, ur[iR].x, ur[iN].x, uW,
                                                      ur[iS].x, ur[iR].y, cg);
                        const double f1 = rhs_point_t(d.x.y, d.y.y, ur[iR].y, ur[iN].y, ur[iR].x,
                                                      ur[iS].y, uE, cg);
                        d.r = make_double2(f0, f1);
                        const bool i0 = !GN || (r >= 1 && r <= n - 1 && in0);
                        const bool i1 = !GN || (r >= 1 && r <= n - 1 && in1);
                        double *row = rhs_next + rowoff(r, ip);
                        if (own(r)) {
                            if (i0 && i1) {
                                st2s(row + c0, d.r);
                            } else {
                                if (i0) row[c0] = f0;
                                if (i1) row[c0 + 1] = f1;
                            }
                        }
                        const double e0 = res_point_t(f0, d.x.x, d.y.x, ur[iR].x, ur[iN].x, uW,
                                                      ur[iS].x, ur[iR].y, cg);
                        const double e1 = res_point_t(f1, d.x.y, d.y.y, ur[iR].y, ur[iN].y,
                                                      ur[iR].x, ur[iS].y, uE, cg);
                        acc2 += (own(r) && i0) ? e0 * e0 : 0.0;
                        acc2 += (own(r) && i1) ? e1 * e1 : 0.0;
                    }
                    to_coef(rd[(q + 1) % NR], cf[(q + 1) % NR]);   // row s+1
#pragma unroll
                    for (int h = 0; h < S; ++h) stage_c(q, h, s + 1 - h);
                    {
                        const int ro = s + 2 - S;
                        st2_ifu(upre + rowoff(ro, ip), c0, own(ro),
                               ur[(q + 2 - S + 2 * NR) % NR]);
                    }
                    if (((q + 1 - S) & 1) == 0) {   // compile-time row parity
                        // residual -> coarse rhs at the even-even points (:73-75)
                        const int r = s + 1 - S;
                        const int iR = (q + 1 - S + 2 * NR) % NR;
                        const int iN = (q - S + 2 * NR) % NR;
                        const int iS = (q + 2 - S + 2 * NR) % NR;
                        const double uW = nbw(ur[iR].y, iR);
                        const bool on = own(r) &&
                                        (!GN || (r >= 1 && r <= n - 2 && in0 && c0 <= n - 2));
                        const double res = res_x(iR, iN, iS, uW);
                        st1_ifu(rhsc + rowoff(r >> 1, ipc), c0 >> 1, on, res);
                    }
                    post_edges(ur, q);
                    if (XG || (p & 1)) __syncthreads();
                    if (p & 1) {
                        it += 2;
                        if (it >= iters) goto done_b;
                    }
                }
            }
        done_b:;
        }
    };

    while (start < end) {
        int strip, a, b;
        region_segment(reg, WPB, pr, start, end, strip, a, b);
        start += b - a;
        // a pair past its region's strips idles on the segment (A and B alike,
        // so each pair's barrier count still matches between its two waves)
        if (__builtin_amdgcn_readfirstlane(strip) >= 0) {
            if (XG) {
                // group g = strips g*WPB .. g*WPB+WPB-1 (regions start at a
                // multiple of WPB, so strip % WPB == pr); the last group is
                // shifted left to end at xend and owns only what is left
                const int g = strip / WPB;
                const int k0 = xg.x0 + g * WGc;
                const int og = g < xg.glast ? k0 : xg.xl;
                march(og - 2 * H + 128 * pr, k0, g < xg.glast ? k0 + WGc : xg.xend, a, b);
            } else {
                march(strip * W - 2 * H, strip * W, strip * W + W, a, b);
            }
        }
    }
    const double tot = wave_sum(acc);   // one partial per wave (A: columns c0, B: c0+1)
    if (l == 0) partials[(long)blockIdx.x * 2 * WPB + wv] = tot;
    if (RS) {
        const double tot2 = wave_sum(acc2);   // B only (A's are +0)
        if (l == 0) partials2[(long)blockIdx.x * 2 * WPB + wv] = tot2;
    }
}

// k_smooth_tile: the same fused pass (K sweeps + optional prolong / restrict
// / norm) for SMALL levels, where the serial row march is latency
// bound.  A workgroup owns a TR x TC output tile and loads it with an EH-wide
// halo (EH = E rounded up to even, so the tile origin has even parity) into
// LDS; all stages then run as parallel colour updates over the whole
// extended tile with one barrier between stages.  The exact region shrinks
// by one point per stage, so the output tile is exact (same argument as
// the row march).  Each lane owns fixed column pairs of the tile and keeps their
// rhs / v1 / v2 in registers for all stages.
// threads per tile workgroup: 1024 (2 pairs per thread, ~80-105 VGPRs)
// against 256 (8 pairs, 155-189 VGPRs): levels 3-7 0.289 -> 0.237 ms per
// cycle (512: 0.248), the stages' per-thread chains being the latency
#ifndef MGX_TILE_THREADS
#define MGX_TILE_THREADS 1024
#endif
template <int K, int MODE, int TRV = 16>
struct TileCfg {
    using C = SmoothCfg<K, MODE>;
    static constexpr int TR = TRV, TC = 64;              // output tile
    static constexpr int EH = (C::E + 1) / 2 * 2;         // halo, even
    static constexpr int RT = TR + 2 * EH, WT = TC + 2 * EH;
    static constexpr int PAIRS = RT * WT / 2;
    static constexpr int THREADS = MGX_TILE_THREADS;
    static constexpr int PPT = (PAIRS + THREADS - 1) / THREADS;   // pairs per thread
};

template <int K, int MODE, int TRV>
__global__ __launch_bounds__(MGX_TILE_THREADS) void k_smooth_tile(
    const double *__restrict__ uin, double *__restrict__ uout, const double *__restrict__ rhs,
    const double *__restrict__ v1, const double *__restrict__ v2, const double *__restrict__ uc,
    long pitchc, double *__restrict__ rhsc, double *__restrict__ partials, int n, long pitch,
    int tiles_x, Coef c, int ra, int rb, int lo, int hi, int xcd) {
    using C = SmoothCfg<K, MODE>;
    using T = TileCfg<K, MODE, TRV>;
    constexpr int S = C::S, EH = T::EH, WT = T::WT, PPT = T::PPT, HW = WT / 2;
    // u of the extended tile split by colour: point (r, col) lives in plane
    // (r + col) & 1 (the tile origin has even parity) at index r*HW + col/2, so
    // a stage's own points and all four neighbours are consecutive 8-B words
    // across consecutive lanes (no LDS bank conflicts; interleaved, the
    // stride-2 accesses were 2-way conflicts on every read)
    __shared__ __attribute__((aligned(16))) double tu[T::RT * WT];
    constexpr int PL = T::PAIRS;   // plane size = RT * WT / 2

    const int t = threadIdx.x;
    int bid = blockIdx.x;
    if (xcd) {   // XCD-contiguous tile order (see wg_order): neighbours' halos share an L2
        const int G = gridDim.x, q = G >> 3, r = G & 7, x = bid & 7;
        bid = x * q + min(x, r) + (bid >> 3);
    }
    const int ty = bid / tiles_x, tx = bid % tiles_x;
    const long i0 = ra + (long)ty * T::TR - EH, j0 = (long)tx * T::TC - EH;   // tile origin (even)
    const int nc = n >> 1;

    // rhs / v1 / v2 of the lane's pairs as scalar arrays (static indices only,
    // so they stay in registers)
    double f0[PPT], f1[PPT], x0[PPT], x1[PPT], y0[PPT], y1[PPT];
    bool ok[PPT];
#pragma unroll
    for (int m = 0; m < PPT; ++m) {
        const int q = t + m * T::THREADS;
        ok[m] = false;
        f0[m] = f1[m] = x0[m] = x1[m] = y0[m] = y1[m] = 0.0;
        if (q >= T::PAIRS) continue;
        const int r = q / HW, k = q % HW;
        const long gi = i0 + r, gj = j0 + 2 * k;
        double2 v = make_double2(0.0, 0.0);
        if (gi >= lo && gi <= hi && gj >= 0 && gj <= n) {
            ok[m] = true;
            const long o = gi * pitch + gj;
            if (!C::ZERO) v = ld2(uin + o);
            if (C::PROL) {
                const long ii = gi >> 1, jj = gj >> 1;
                const double *p0 = uc + ii * pitchc + jj;
                const double q00 = p0[0], q01 = (jj + 1 <= nc) ? p0[1] : 0.0;
                double2 pr;
                if (!(gi & 1)) {
                    pr.x = q00;
                    pr.y = (q00 + q01) / 2;
                } else {
                    const double q10 = p0[pitchc], q11 = (jj + 1 <= nc) ? p0[pitchc + 1] : 0.0;
                    pr.x = (q00 + q10) / 2;
                    pr.y = (q00 + q10 + q01 + q11) / 4;
                }
                v.x = v.x + pr.x;
                v.y = v.y + pr.y;
            }
            const double2 rr = ld2(rhs + o), xx = ld2(v1 + o), yy = ld2(v2 + o);
            f0[m] = rr.x;
            f1[m] = rr.y;
            x0[m] = xx.x;
            x1[m] = xx.y;
            y0[m] = yy.x;
            y1[m] = yy.y;
        }
        tu[(r & 1) * PL + q] = v.x;   // q = r*HW + k
        tu[((r & 1) ^ 1) * PL + q] = v.y;
    }
    // per pair, once: its LDS index, row parity and which of its two points
    // the stages may update (interior of the level and of the extended tile);
    // the stage loop then does no index arithmetic
    int xs[PPT];
    unsigned upd = 0, rpar = 0;   // bits 2m / 2m+1: column 2k / 2k+1 updatable; bit m: row odd
#pragma unroll
    for (int m = 0; m < PPT; ++m) {
        const int q = t + m * T::THREADS;
        xs[m] = 0;
        if (q >= T::PAIRS || !ok[m]) continue;
        const int r = q / HW, k = q % HW;
        const long gi = i0 + r;
        xs[m] = q;   // r*HW + k
        rpar |= (unsigned)(r & 1) << m;
#pragma unroll
        for (int cs = 0; cs < 2; ++cs) {
            const long gj = j0 + 2 * k + cs;
            if (gi >= 1 && gi <= n - 1 && gj >= 1 && gj <= n - 1 && r >= 1 && r <= T::RT - 2 &&
                2 * k + cs >= 1 && 2 * k + cs <= WT - 2)
                upd |= 1u << (2 * m + cs);
        }
    }
    __syncthreads();

#pragma unroll
    for (int h = 0; h < S; ++h) {
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            const int q = t + m * T::THREADS;
            if (q >= T::PAIRS) continue;
            const int cs = (int)((rpar >> m) & 1u) ^ (h & 1);   // origin parity is even
            if (!((upd >> (2 * m + cs)) & 1u)) continue;
            const int b = xs[m];
            double *own = tu + (h & 1) * PL;           // colour being updated
            const double *oth = tu + ((h & 1) ^ 1) * PL;   // its neighbours
            const double fr = cs ? f1[m] : f0[m], fx = cs ? x1[m] : x0[m],
                         fy = cs ? y1[m] : y0[m];
            own[b] = gs_point_fast(fr, fx, fy, oth[b - HW], oth[b - 1 + cs], oth[b + HW],
                                   oth[b + cs], c);
        }
        __syncthreads();
    }

    double acc = 0.0;
#pragma unroll
    for (int m = 0; m < PPT; ++m) {
        const int q = t + m * T::THREADS;
        if (q >= T::PAIRS || !ok[m]) continue;
        const int r = q / HW, k = q % HW;
        if (r < EH || r >= EH + T::TR || 2 * k < EH || 2 * k >= EH + T::TC) continue;
        const long gi = i0 + r, gj = j0 + 2 * k;
        if (gi >= rb) continue;
        const double *p0 = tu + (r & 1) * PL, *p1 = tu + ((r & 1) ^ 1) * PL;
        const int b = q;   // r*HW + k; column 2k in p0, 2k+1 in p1
        st2(uout + gi * pitch + gj, make_double2(p0[b], p1[b]));
        if (C::REST || C::NORM) {
            const bool in0 = gi >= 1 && gi <= n - 1 && gj >= 1 && gj <= n - 1;
            const bool in1 = gi >= 1 && gi <= n - 1 && gj + 1 <= n - 1;
            if (C::REST) {
                if (!(gi & 1) && in0 && gi <= n - 2 && gj <= n - 2)
                    rhsc[(gi >> 1) * pitchc + (gj >> 1)] =
                        res_point(f0[m], x0[m], y0[m], p0[b], p1[b - HW], p1[b - 1], p1[b + HW],
                                  p1[b], c);
            } else {
                if (in0) {
                    const double res = res_point(f0[m], x0[m], y0[m], p0[b], p1[b - HW],
                                                 p1[b - 1], p1[b + HW], p1[b], c);
                    acc += res * res;
                }
                if (in1) {
                    const double res = res_point(f1[m], x1[m], y1[m], p1[b], p0[b - HW],
                                                 p0[b], p0[b + HW], p0[b + 1], c);
                    acc += res * res;
                }
            }
        }
    }
    if (C::NORM) {
        __shared__ double red_lds[T::THREADS / 64];
        const double tot = block_sum(acc, red_lds);
        if (t == 0) partials[bid] = tot;
    }
}

// k_xtile: the cross-cycle pass of k_xsmooth as 2-D LDS tiles, for the edge
// regions of a SHORT row block (a multi-GPU rank's two boundary strips and
// its top / bottom bands) and for short row ranges (the bands of the
// overlapped exchange).  There the guarded row march is latency bound: every
// workgroup pays a ~40-row warm-up on a short segment, one dependent row step
// after another (~0.15 ms whatever the block height), while a tile runs all
// its stages on all its rows at once (the cost grows with the rows instead:
// on a whole 16384-row level the march stays faster).
//
// A workgroup owns a TR x 64 output tile and loads it with an EH-point halo
// (EH = E rounded up to even, E = the stages of the pass plus its residual
// stage) into LDS, split by colour: point (r, col) of the extended tile lives
// in plane (r + col) & 1 at index r*HW + col/2, so a stage's own points and
// all four neighbours are consecutive 8-B words across consecutive lanes (no
// bank conflicts).  Stages run as parallel colour updates with one barrier
// between them; the exact region shrinks by one point per stage, so the
// owned points are exact (EH >= E).
//
// Thread map: threads 0..127 own column pairs of the even rows, 128..255 of
// the odd rows, so in every stage each thread updates the same point of each
// of its pairs (x = column 2k on even-parity stages of even rows, ...) and
// all its operands sit at compile-time indices: each pair keeps the rhs and
// the four coefficients (gs.cpp:126-129) of its two points, computed once
// from v1 / v2 at load instead of in every stage.  The same expressions as
// gs_point, so every value is bitwise the reference's.
//
// The pass: S stages of the post-smoothing of cycle k from uin + P(uc)
// (gs.cpp:238-265), the residual norm of u_post (multigrid.cpp:112-113, one
// partial per tile) and the optional u_post store, S stages of the
// pre-smoothing of cycle k+1, the u_pre store and the residual at the
// even-even points -> coarse rhs (multigrid.cpp:73-75).
// Owned regions: up to 4 rectangles of columns [c0, c1) x rows [r0, r1),
// each cut into TR x 64 tiles from (r0 & ~1, c0 & ~1) (even tile origins:
// the planes are the global colours); a tile owns its points inside its
// rectangle.
struct TileRegions {
    int c0[4], c1[4], r0[4], r1[4];
    int tx[4];     // tiles per tile row of region k
    int pre[5];    // prefix tile counts
    int count;
};

template <int K, int TRV>
struct XTileCfg {
    static constexpr int S = 2 * K;
    static constexpr int E = 2 * S + 1;   // both halves + the restriction residual
    static constexpr int EH = (E + 1) / 2 * 2;
    static constexpr int TR = TRV, TC = 64;
    static constexpr int RT = TR + 2 * EH, WT = TC + 2 * EH, HW = WT / 2;
    static constexpr int PL = RT * HW;              // plane size (doubles)
    static constexpr int HALF = (RT / 2) * HW;      // pairs of one row parity
    static constexpr int PPT = (HALF + 127) / 128;  // pairs per thread
};

// rhs and coefficients of one point: (rhs - cn*uN - cw*uW - cs*uS - ce*uE) / d
struct PtCoef {
    double f, cn, cw, cs, ce;
};

template <int K, int TRV>
__global__ __launch_bounds__(256) void k_xtile(
    const double *__restrict__ uin, double *__restrict__ uout, double *__restrict__ upost,
    const double *__restrict__ rhs, const double *__restrict__ v1, const double *__restrict__ v2,
    const double *__restrict__ uc, long pitchc, double *__restrict__ rhsc,
    double *__restrict__ partials, int n, long pitch, TileRegions reg, Coef c, int lo, int hi,
    int store_post) {
    using T = XTileCfg<K, TRV>;
    constexpr int S = T::S, EH = T::EH, WT = T::WT, RT = T::RT, PPT = T::PPT, HW = T::HW;
    constexpr int PL = T::PL, HALF = T::HALF;
    __shared__ __attribute__((aligned(16))) double tu[2 * PL];
    __shared__ double red_lds[4];

    const int t = threadIdx.x;
    const int bid = blockIdx.x;
    int k = 0;
    while (k + 1 < reg.count && bid >= reg.pre[k + 1]) ++k;
    const int loc = bid - reg.pre[k];
    const int ty = loc / reg.tx[k], tx = loc % reg.tx[k];
    const int R0 = (reg.r0[k] & ~1) + ty * T::TR, C0 = (reg.c0[k] & ~1) + tx * T::TC;
    const int oa = max(R0, reg.r0[k]), ob = min(R0 + T::TR, reg.r1[k]);   // owned rows
    const int ca = max(C0, reg.c0[k]), cb = min(C0 + T::TC, reg.c1[k]);   // owned columns
    const long i0 = R0 - EH, j0 = C0 - EH;   // tile origin (even, even)
    const int nc = n >> 1;
    const int par = t >> 7;   // row parity of this thread's pairs (wave-uniform)
    const int u = t & 127;

    // pair m: LDS index q[m]; P0[m] = the point updated on even stages (column
    // 2k + par), P1[m] the other; bits: 2m / 2m+1 updatable, 2m+... owned
    int qi[PPT];
    PtCoef P0[PPT], P1[PPT];
    unsigned upd = 0, own = 0;
#pragma unroll
    for (int m = 0; m < PPT; ++m) {
        const int j = u + m * 128;
        qi[m] = 0;
        P0[m] = P1[m] = PtCoef{0.0, 0.0, 0.0, 0.0, 0.0};
        if (j >= HALF) continue;
        const int r = 2 * (j / HW) + par, kk = j % HW;
        const int q = r * HW + kk;
        qi[m] = q;
        const long gi = i0 + r, gj = j0 + 2 * kk;
        double2 v = make_double2(0.0, 0.0);
        if (gi >= lo && gi <= hi && gj >= 0 && gj <= n) {
            const long o = gi * pitch + gj;
            v = ld2(uin + o);
            {
                const long ii = gi >> 1, jj = gj >> 1;
                const double *p0 = uc + ii * pitchc + jj;
                const double q00 = p0[0], q01 = (jj + 1 <= nc) ? p0[1] : 0.0;
                double2 pr;
                if (!(gi & 1)) {
                    pr.x = q00;
                    pr.y = (q00 + q01) / 2;
                } else {
                    const double q10 = p0[pitchc], q11 = (jj + 1 <= nc) ? p0[pitchc + 1] : 0.0;
                    pr.x = (q00 + q10) / 2;
                    pr.y = (q00 + q10 + q01 + q11) / 4;
                }
                v.x = v.x + pr.x;
                v.y = v.y + pr.y;
            }
            const double2 rr = ld2(rhs + o), xx = ld2(v1 + o), yy = ld2(v2 + o);
            // gs.cpp:126-129: aa, bb from v2 (W / E), cc, dd from v1 (N / S)
            const PtCoef X{rr.x, coef_a(xx.x, c), coef_a(yy.x, c), coef_b(xx.x, c), coef_b(yy.x, c)};
            const PtCoef Y{rr.y, coef_a(xx.y, c), coef_a(yy.y, c), coef_b(xx.y, c), coef_b(yy.y, c)};
            P0[m] = par ? Y : X;
            P1[m] = par ? X : Y;
#pragma unroll
            for (int cs = 0; cs < 2; ++cs) {   // cs: column 2kk + cs
                if (gi >= 1 && gi <= n - 1 && gj + cs >= 1 && gj + cs <= n - 1 && r >= 1 &&
                    r <= RT - 2 && 2 * kk + cs >= 1 && 2 * kk + cs <= WT - 2)
                    upd |= 1u << (2 * m + (cs ^ par));   // bit 2m: even stages
            }
            if (gi >= oa && gi < ob && gj >= ca && gj < cb) own |= 1u << m;
        }
        tu[par * PL + q] = v.x;          // column 2kk: plane r & 1 = par
        tu[(par ^ 1) * PL + q] = v.y;
    }
    __syncthreads();

    // stages [h0, h1): stage h updates plane h & 1; this thread's point of
    // pair m there is column 2k + cs, cs = par ^ (h & 1): W = q-1+cs, E = q+cs
    auto stages = [&](const int h0, const int h1) {
#pragma unroll
        for (int h = h0; h < h1; ++h) {
            const int cs = par ^ (h & 1);
            double *ow = tu + (h & 1) * PL;
            const double *ot = tu + ((h & 1) ^ 1) * PL;
#pragma unroll
            for (int m = 0; m < PPT; ++m) {
                if (!((upd >> (2 * m + (h & 1))) & 1u)) continue;
                const int q = qi[m];
                const PtCoef &P = (h & 1) ? P1[m] : P0[m];
                const double uN = ot[q - HW], uS = ot[q + HW];
                const double uW = ot[q - 1 + cs], uE = ot[q + cs];
                ow[q] = div_diag(P.f - P.cn * uN - P.cw * uW - P.cs * uS - P.ce * uE, c);
            }
            __syncthreads();
        }
    };
    // residual of this thread's point (even-stage point e = 1: P0, else P1) of pair m
    auto residual = [&](const int m, const bool even_pt) -> double {
        const int q = qi[m];
        const int cs = even_pt ? par : par ^ 1;      // column 2k + cs
        const int pl = even_pt ? 0 : 1;              // its plane
        const double *pu = tu + pl * PL, *ot = tu + (pl ^ 1) * PL;
        const PtCoef &P = even_pt ? P0[m] : P1[m];
        // gs.cpp:75: rhs - (d*u + cc*uN + aa*uW + dd*uS + bb*uE)
        return P.f - (c.dgs * pu[q] + P.cn * ot[q - HW] + P.cw * ot[q - 1 + cs] +
                      P.cs * ot[q + HW] + P.ce * ot[q + cs]);
    };
    auto gidx = [&](const int m, long &gi, long &gj) {
        const int r = qi[m] / HW, kk = qi[m] % HW;
        gi = i0 + r;
        gj = j0 + 2 * kk;
    };
    // owned pairs -> dst (column 2k lives in plane par, 2k+1 in the other)
    auto store = [&](double *dst) {
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            if (!((own >> m) & 1u)) continue;
            long gi, gj;
            gidx(m, gi, gj);
            const int q = qi[m];
            st2(dst + gi * pitch + gj, make_double2(tu[par * PL + q], tu[(par ^ 1) * PL + q]));
        }
    };
    // sum of squares of the residual over the owned interior points
    auto norm_acc = [&]() -> double {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            if (!((own >> m) & 1u)) continue;
            long gi, gj;
            gidx(m, gi, gj);
            if (gi < 1 || gi > n - 1) continue;
            // the even-stage point (column 2k + par), then the other; static
            // operand indices (a runtime choice would put P0 / P1 in scratch)
            const bool okx = gj >= 1 && gj <= n - 1, oky = gj + 1 <= n - 1;
            const double re = residual(m, true), ro = residual(m, false);
            acc += (par ? oky : okx) ? re * re : 0.0;
            acc += (par ? okx : oky) ? ro * ro : 0.0;
        }
        return acc;
    };

    stages(0, S);   // post-smoothing of cycle k
    if (store_post) store(upost);
    const double acc = norm_acc();
    __syncthreads();
    stages(S, 2 * S);   // pre-smoothing of cycle k+1
    store(uout);
    if (par == 0) {   // even rows: residual -> coarse rhs at the even-even points
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            if (!((own >> m) & 1u)) continue;
            long gi, gj;
            gidx(m, gi, gj);
            if (gi < 1 || gi > n - 2 || gj < 1 || gj > n - 2) continue;
            rhsc[(gi >> 1) * pitchc + (gj >> 1)] = residual(m, true);   // column 2k
        }
    }
    const double tot = block_sum(acc, red_lds);
    if (t == 0) partials[bid] = tot;
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
__global__ __launch_bounds__(1024) void k_coarse_solve(double *u, const double *rhs,
                                                       const double *v1, const double *v2,
                                                       int n, long pitch, Coef c, double tol,
                                                       int maxit, int zero_first,
                                                       double *stats) {
    __shared__ double lds[16];
    __shared__ double s_norm;
    const int t = threadIdx.x;
    // 64 x 16 threads: lane tx walks the columns, ty the rows (no integer
    // division in the loops: 64-bit div/mod is a long emulated sequence)
    const int tx = t & 63, ty = t >> 6;
    if (zero_first) {
        for (long p = t; p < (long)(n + 1) * pitch; p += 1024) u[p] = 0.0;
        __syncthreads();
    }
    int it = 0;
    double res = 1.0;
    while (it < maxit && res > tol) {
        for (int colour = 0; colour < 2; ++colour) {
            for (int i = 1 + ty; i <= n - 1; i += 16) {
                // first column of this colour in row i: (i + j) & 1 == colour
                const int jc = 1 + ((i + 1 + colour) & 1);
                for (int j = jc + 2 * tx; j <= n - 1; j += 128) {
                    const long p = (long)i * pitch + j;
                    u[p] = gs_point(rhs[p], v1[p], v2[p], u[p - pitch], u[p - 1], u[p + pitch],
                                    u[p + 1], c);
                }
            }
            __syncthreads();
        }
        double acc = 0.0;
        for (int i = 1 + ty; i <= n - 1; i += 16)
            for (int j = 1 + tx; j <= n - 1; j += 64) {
                const long p = (long)i * pitch + j;
                const double r = res_point(rhs[p], v1[p], v2[p], u[p], u[p - pitch], u[p - 1],
                                           u[p + pitch], u[p + 1], c);
                acc += r * r;
            }
        double s = block_sum(acc, lds);
        if (t == 0) s_norm = sqrt(s);
        __syncthreads();
        res = s_norm;
        ++it;
        __syncthreads();
    }
    if (t == 0) {
        stats[0] += it;
        stats[1] = res;
    }
}

// The same solve with u, rhs, v1, v2 held in LDS (n <= 64: 4 x 65^2 doubles
// = 135 KB of the CU's 160 KB): the loop's loads and stores are LDS accesses
// instead of L2 round trips.  Same sweep order, term order and reduction
// order as k_coarse_solve, so u, the norms and the iteration count are
// bitwise those of k_coarse_solve.
constexpr int kCoarseLdsMaxN = 64;
__global__ __launch_bounds__(1024) void k_coarse_solve_lds(double *u, const double *rhs,
                                                           const double *v1, const double *v2,
                                                           int n, long pitch, Coef c, double tol,
                                                           int maxit, int zero_first,
                                                           double *stats) {
    constexpr int NP = kCoarseLdsMaxN + 1;
    constexpr int SZ = NP * NP;
    __shared__ double su[SZ], sr[SZ], sx[SZ], sy[SZ];
    __shared__ double lds[16];
    __shared__ double s_norm;
    const int t = threadIdx.x;
    const int tx = t & 63, ty = t >> 6;
    if (zero_first)
        for (long p = t; p < (long)(n + 1) * pitch; p += 1024) u[p] = 0.0;
    for (int i = ty; i <= n; i += 16)
        for (int j = tx; j <= n; j += 64) {
            const long p = (long)i * pitch + j;
            const int q = i * NP + j;
            su[q] = zero_first ? 0.0 : u[p];
            sr[q] = rhs[p];
            sx[q] = v1[p];
            sy[q] = v2[p];
        }
    __syncthreads();
    int it = 0;
    double res = 1.0;
    while (it < maxit && res > tol) {
        for (int colour = 0; colour < 2; ++colour) {
            for (int i = 1 + ty; i <= n - 1; i += 16) {
                const int jc = 1 + ((i + 1 + colour) & 1);
                for (int j = jc + 2 * tx; j <= n - 1; j += 128) {
                    const int q = i * NP + j;
                    su[q] = gs_point(sr[q], sx[q], sy[q], su[q - NP], su[q - 1], su[q + NP],
                                     su[q + 1], c);
                }
            }
            __syncthreads();
        }
        double acc = 0.0;
        for (int i = 1 + ty; i <= n - 1; i += 16)
            for (int j = 1 + tx; j <= n - 1; j += 64) {
                const int q = i * NP + j;
                const double r = res_point(sr[q], sx[q], sy[q], su[q], su[q - NP], su[q - 1],
                                           su[q + NP], su[q + 1], c);
                acc += r * r;
            }
        double s = block_sum(acc, lds);
        if (t == 0) s_norm = sqrt(s);
        __syncthreads();
        res = s_norm;
        ++it;
        __syncthreads();
    }
    for (int i = 1 + ty; i <= n - 1; i += 16)
        for (int j = 1 + tx; j <= n - 1; j += 64) u[(long)i * pitch + j] = su[i * NP + j];
    if (t == 0) {
        stats[0] += it;
        stats[1] = res;
    }
}

inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }

}  // namespace

// ------------------------------------------------------------------ launchers
#define MGX_LAUNCH(kern, grid, block, s, ...) \
    hipLaunchKernelGGL((kern), (grid), (block), 0, (s), __VA_ARGS__)

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

long g_xfast = 1;   // unguarded interior march kernels (tuning key "xfast")
void set_xfast(long v) { g_xfast = v; }
long get_xfast() { return g_xfast; }

template <int WPB>
static void add_region(MarchRegions &r, int sfirst, int slim, int r0, int r1) {
    if (slim <= sfirst || r1 <= r0) return;
    const int k = r.count++;
    r.sfirst[k] = sfirst;
    r.slim[k] = slim;
    r.r0[k] = r0;
    r.r1[k] = r1;
    r.pre[k + 1] = r.pre[k] + (long)((slim - sfirst + WPB - 1) / WPB) * (r1 - r0);
}

// Split a march over strips of width W (halo H pairs) and rows [ra, rb) into
// the unguarded kernel's work -- interior strips (every lane a column in
// [1, n-1]) x rows [TOP, n+1-BOT) -- and the guarded kernel's: the boundary
// strips and the top / bottom bands (~1-2 % of the points).
// interior strips [si0, si1) (every lane a column in [1, n-1]) and the rows
// [ma, mb) of [ra, rb) an unguarded march may own
static void march_split(long n, int W, int H, int ra, int rb, int top, int bot, int &si0,
                        int &si1, int &ma, int &mb) {
    const int strips = (int)((n + 1 + W - 1) / W);
    si0 = strips;
    si1 = 0;
    for (int st = 0; st < strips; ++st) {
        const long c_first = (long)st * W - 2 * H, c_last = c_first + 127;
        if (c_first >= 1 && c_last <= n - 1) {
            si0 = std::min(si0, st);
            si1 = st + 1;
        }
    }
    ma = std::max(ra, top);
    mb = std::min(rb, (int)n + 1 - bot);
}

template <int WPB>
static void march_regions(long n, int W, int H, int ra, int rb, int top, int bot, bool split,
                          MarchRegions &inner, MarchRegions &edge) {
    inner = MarchRegions{};
    edge = MarchRegions{};
    const int strips = (int)((n + 1 + W - 1) / W);
    int si0, si1, ma, mb;
    march_split(n, W, H, ra, rb, top, bot, si0, si1, ma, mb);
    if (split && si1 > si0 && mb > ma) {
        add_region<WPB>(inner, si0, si1, ma, mb);
        add_region<WPB>(edge, 0, si0, ra, rb);
        add_region<WPB>(edge, si1, strips, ra, rb);
        add_region<WPB>(edge, si0, si1, ra, ma);
        add_region<WPB>(edge, si0, si1, mb, rb);
    } else {
        add_region<WPB>(edge, 0, strips, ra, rb);
    }
}

long g_march_min_rows = 32;   // fewest rows per workgroup of a wave march (tuning key)
static long march_min_rows() { return g_march_min_rows; }
void set_march_min_rows(long v) { g_march_min_rows = v; }
long get_march_min_rows() { return g_march_min_rows; }

long g_march_order = -1;   // tuning key "march_order": bit 0 bands, bit 1 XCD order
static long march_order() {
    if (g_march_order < 0) {
        const char *e = getenv("MGX_MARCH_ORDER");
        g_march_order = e ? atol(e) : 3;
    }
    return g_march_order;
}
void set_march_order(long v) { g_march_order = v; }
long get_march_order() { return march_order(); }

// The work order of a launch of `upw` units per workgroup (march_order):
// band-major with bands of upw rows on a one-region launch, and/or the
// XCD-contiguous workgroup order.  Only the order changes, not the work.
// Measured (N=16384, per cycle): cross pass 2.92 -> 2.78 ms, level 1 1.13 ->
// 1.11 ms; with ~80-row segments (level 2) bands cost +12 %, so they apply
// from kBandMinRows rows per workgroup.
constexpr long kBandMinRows = 192;
static MarchRegions order_regions(const MarchRegions &reg, long upw) {
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
static unsigned plan_march(const MarchRegions &reg, int wpb, long slots, long min_rows,
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

template <int WPB, int K, int MODE, bool G, bool PD>
static int wsmooth_launch_pd(const SmoothArgs &A, const MarchRegions &reg, double *partials,
                             long max_wgs, hipStream_t s) {
    const long total = reg.pre[reg.count];
    if (total <= 0) return 0;
    static int slots = 0;   // resident workgroups of this instantiation
    if (!slots) {
        int dev = 0, cus = 0, per = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_wsmooth<WPB, K, MODE, G, PD>,
                                                           64 * WPB, 0);
        slots = std::max(1, cus) * std::max(1, per);
    }
    long upw;
    MarchRegions r;
    // one segment per workgroup when the last band is short (warm-up ~E + NR/2
    // rows: the prologue aligns the first step to NR): level 1 at N=16384
    // 1.11 -> 1.075 ms (its 19 last-band workgroups each marched pieces of two
    // strips); the same per rank on 8 row blocks
    const unsigned grid = plan_march(reg, WPB, slots, march_min_rows(), max_wgs,
                                     WCfg<K, MODE>::E + WCfg<K, MODE>::NR / 2, upw, r);
    MGX_LAUNCH((k_wsmooth<WPB, K, MODE, G, PD>), dim3(grid), dim3(64 * WPB), s, A.uin, A.uout,
               A.rhs, A.v1, A.v2, A.uc, A.pitchc, A.rhsc, partials, (int)A.n, A.pitch, r, upw,
               A.c, A.lo, A.hi, A.rhs_out, A.zrow ? A.zrow : A.v1, A.zrow ? A.vz : 0x7fffffff);
    return (int)grid * WPB;   // NORM partials written
}
// the short division when the diagonal is positive (every nu <= 0)
template <int WPB, int K, int MODE, bool G>
static int wsmooth_launch(const SmoothArgs &A, const MarchRegions &reg, double *partials,
                          long max_wgs, hipStream_t s) {
    if (A.c.dgs > 0) return wsmooth_launch_pd<WPB, K, MODE, G, true>(A, reg, partials, max_wgs, s);
    return wsmooth_launch_pd<WPB, K, MODE, G, false>(A, reg, partials, max_wgs, s);
}

// One guarded launch over the whole level.  (The interior / edge split that
// pays for k_xsmooth measured -5 % on the unguarded kernels of levels 1-2 and
// +40 % for the edge launches: their passes are only ~300 rows per workgroup,
// so the edge warm-ups do not amortise.)
template <int WPB, int K, int MODE>
static int smooth_winst(const SmoothArgs &A, hipStream_t s) {
    using C = WCfg<K, MODE>;
    MarchRegions inner, edge;
    march_regions<WPB>(A.n, C::W, C::H, A.ra, A.rb, C::TOP, C::BOT, false, inner, edge);
    return wsmooth_launch<WPB, K, MODE, true>(A, edge, A.partials, kNormBlocks / WPB, s);
}


template <int WPB, int K, bool G, bool RS = false, bool SV = false, bool XG = false>
static int xsmooth_slots() {
    static int slots = 0;   // resident workgroups of this instantiation
    if (!slots) {
        int dev = 0, cus = 0, per = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per,
                                                           k_xsmooth<WPB, K, G, RS, SV, XG>,
                                                           128 * WPB, 0);
        slots = std::max(1, cus) * std::max(1, per);
    }
    return slots;
}

// One launch over `reg`; min_rows: the fewest rows per workgroup (each
// workgroup's march pays a warm-up of ~EA + EB + D rows).  Returns the norm
// partials written (grid * 2 * WPB: one per wave) at `partials`.  geo: the
// group geometry (XG) or the guarded kernel's excluded rectangle.
template <int WPB, int K, bool G, bool RS, bool SV, bool XG>
static int xsmooth_launch_sv(const XArgs &A, const MarchRegions &reg, double *partials, int lo,
                             int hi, long min_rows, long max_wgs, const XGeo &geo,
                             hipStream_t s) {
    const long total = reg.pre[reg.count];
    if (total <= 0) return 0;
    long upw;
    MarchRegions r;
    using X = XCfg<K>;
    const unsigned grid = plan_march(reg, WPB, xsmooth_slots<WPB, K, G, RS, SV, XG>(), min_rows,
                                     max_wgs, X::EA + X::EB + X::D + X::NR / 2, upw, r);
    // RS: the second partials (the next step's initial norm) at the same
    // offsets, kNormBlocks further on
    MGX_LAUNCH((k_xsmooth<WPB, K, G, RS, SV, XG>), dim3(grid), dim3(128 * WPB), s, A.uin,
               A.upost, A.upre, A.rhs, A.v1, A.v2, A.uc, A.pitchc, A.rhsc, partials, (int)A.n,
               A.pitch, r, upw, A.c, lo, hi, A.store_post ? 1 : 0, A.rhs_next,
               RS ? partials + kNormBlocks : (double *)nullptr, A.sa1, A.sb1, A.sa2, A.sb2, geo);
    return (int)grid * 2 * WPB;
}
// SV when the level's velocity factors are given (XArgs::sa1)
template <int WPB, int K, bool G, bool RS = false, bool XG = false>
static int xsmooth_launch(const XArgs &A, const MarchRegions &reg, double *partials, int lo, int hi,
                          long min_rows, long max_wgs, hipStream_t s,
                          const XGeo &geo = XGeo{0, 0, 0, 0, 0, 0, 0, 0}) {
    if (A.sa1 && A.sb1 && A.sa2 && A.sb2)
        return xsmooth_launch_sv<WPB, K, G, RS, true, XG>(A, reg, partials, lo, hi, min_rows,
                                                          max_wgs, geo, s);
    return xsmooth_launch_sv<WPB, K, G, RS, false, XG>(A, reg, partials, lo, hi, min_rows,
                                                       max_wgs, geo, s);
}

// tuning key "xgroup": the group-exchange interior kernel (XG), default off:
// bitwise, 13 % less VALU per owned point (28 halo columns per 512 instead of
// per 128), but level 0 2.09 vs 1.88 ms at N=16384 -- the per-step barrier
// and the exchange reads' LDS latency on every stage chain (at 250 VGPRs the
// reads cannot be issued ahead) cost more than the halo work saved
long g_xgroup = 0;
void set_xgroup(long v) { g_xgroup = v; }
long get_xgroup() { return g_xgroup; }

// The XG launch's work: groups of WPB strips, each owning WGc = 128 WPB - 4H
// columns, group 0 from column x0 = 2H + 2 (lane 0 on column 2, even), the
// last group shifted left so that its last lane is column n-1 (owning what
// the others leave up to xend), x rows [ma, mb); and the guarded kernel's
// work around it in W-column strips: the strips holding columns [0, x0) and
// [xend, n] on all rows, the others on the rows outside [ma, mb), with the
// XG launch's rectangle excluded (XGeo::ec0..er1).  false: no group fits.
template <int WPB, int K>
static bool xg_regions(long n, int ra, int rb, int top, int bot, MarchRegions &inner,
                       MarchRegions &edge, XGeo &geo) {
    using X = XCfg<K>;
    // the XG march starts 2 rows earlier (k_xsmooth): 2 more margin rows
    const int ma = std::max(ra, top + 2), mb = std::min(rb, (int)n + 1 - bot);
    constexpr int H = X::H, W = X::W, WGc = 128 * WPB - 4 * H;
    inner = MarchRegions{};
    edge = MarchRegions{};
    const int x0 = 2 * H + 2;
    const long xl = (n + 2 * H - 128 * WPB) & ~1L;
    if (xl < x0 || mb <= ma) return false;
    const int xend = (int)xl + WGc;
    const int groups = (xend - x0 + WGc - 1) / WGc;
    geo = XGeo{x0, (int)xl, xend, groups - 1, x0, xend, ma, mb};
    add_region<WPB>(inner, 0, groups * WPB, ma, mb);
    const int strips = (int)((n + 1 + W - 1) / W);
    const int sl = (x0 + W - 1) / W, sr = std::min(strips, xend / W);
    add_region<1>(edge, 0, sl, ra, rb);
    add_region<1>(edge, sr, strips, ra, rb);
    add_region<1>(edge, sl, sr, ra, ma);
    add_region<1>(edge, sl, sr, mb, rb);
    return true;
}

static void add_tile_region(TileRegions &r, int c0, int c1, int r0, int r1, int TR) {
    if (c1 <= c0 || r1 <= r0) return;
    const int k = r.count++;
    r.c0[k] = c0;
    r.c1[k] = c1;
    r.r0[k] = r0;
    r.r1[k] = r1;
    r.tx[k] = (c1 - (c0 & ~1) + 63) / 64;
    const int ty = (r1 - (r0 & ~1) + TR - 1) / TR;
    r.pre[k + 1] = r.pre[k] + r.tx[k] * ty;
}

// Row blocks of at most this many rows run the cross pass's edges as tiles
// (tuning key "xtile_max_rows"; 0 = never); row ranges too short for the
// unguarded march (< kXTileAllRows rows between its margins) run entirely as
// tiles.
long g_xtile_max_rows = 4097;
void set_xtile_max_rows(long v) { g_xtile_max_rows = v; }
long get_xtile_max_rows() { return g_xtile_max_rows; }
constexpr int kXTileAllRows = 96;
constexpr int kXTileRows = 16;

// The cross pass of a short row block: the unguarded march over the interior
// strips x rows [ma, mb), k_xtile over the boundary strips and the top /
// bottom bands (or over everything, when [ma, mb) is short).
// the unguarded march's row margins, widened by the split pass's bands
template <int K>
static void xmargins(const XArgs &A, int ra, int rb, int &top, int &bot) {
    using X = XCfg<K>;
    top = std::max(X::TOP, ra + A.band);
    bot = std::max(X::BOT, (int)A.n + 1 - rb + A.band);
}

template <int WPB, int K>
static int xsmooth_tiled(const XArgs &A, int ra, int rb, int lo, int hi, hipStream_t s) {
    using X = XCfg<K>;
    const long n = A.n;
    int si0, si1, ma, mb, top, bot;
    xmargins<K>(A, ra, rb, top, bot);
    march_split(n, X::W, X::H, ra, rb, top, bot, si0, si1, ma, mb);
    TileRegions t{};
    MarchRegions ginner, gedge;
    XGeo geo{};
    const bool xg = g_xgroup != 0 && xg_regions<WPB, K>(n, ra, rb, top, bot, ginner, gedge, geo);
    if (xg) ma = geo.er0;   // the XG march's rows: [er0, er1)
    const bool inner_march = (xg || si1 > si0) && mb - ma >= kXTileAllRows;
    if (inner_march) {
        const int ca = xg ? geo.x0 : si0 * X::W;
        const int cb = xg ? geo.xend : (int)std::min<long>(n + 1, (long)si1 * X::W);
        add_tile_region(t, 0, ca, ra, rb, kXTileRows);
        add_tile_region(t, cb, (int)n + 1, ra, rb, kXTileRows);
        add_tile_region(t, ca, cb, ra, ma, kXTileRows);
        add_tile_region(t, ca, cb, mb, rb, kXTileRows);
    } else {
        add_tile_region(t, 0, (int)n + 1, ra, rb, kXTileRows);
    }
    const int tiles = t.pre[t.count];
    // one norm partial per tile; the inner march writes at most kNormBlocks / 2
    if (tiles > kNormBlocks / 2) return -2;   // too many: the caller marches the edges
    int pm = A.phase == 2 ? A.partials_done : 0;
    if (inner_march && A.phase != 2) {
        if (xg) {
            pm = xsmooth_launch<WPB, K, false, false, true>(A, ginner, A.partials, lo, hi,
                                                            A.min_rows,
                                                            kNormBlocks / (2 * WPB) / 2, s, geo);
        } else {
            MarchRegions inner{};
            add_region<WPB>(inner, si0, si1, ma, mb);
            pm = xsmooth_launch<WPB, K, false>(A, inner, A.partials, lo, hi, A.min_rows,
                                               kNormBlocks / (2 * WPB) / 2, s);
        }
    }
    if (A.phase == 1) return pm;
    if (tiles > 0)
        MGX_LAUNCH((k_xtile<K, kXTileRows>), dim3((unsigned)tiles), dim3(256), s, A.uin, A.upre,
                   A.upost, A.rhs, A.v1, A.v2, A.uc, A.pitchc, A.rhsc, A.partials + pm, (int)n,
                   A.pitch, t, A.c, lo, hi, A.store_post ? 1 : 0);
    return pm + tiles;
}

// The cross pass as two launches: the unguarded kernel over the interior
// strips x rows [TOP, n+1-BOT), the guarded one over the rest (boundary
// strips, top / bottom bands: ~1.7 % of the points at N=16384).
template <int WPB, int K>
static int xsmooth_inst(const XArgs &A, hipStream_t s) {
    using X = XCfg<K>;
    const long n = A.n;
    int ra = A.ra, rb = A.rb, lo = A.lo, hi = A.hi;
    if (rb < 0) {
        ra = 0;
        rb = (int)n + 1;
        lo = 0;
        hi = (int)n;
    }
    if (A.rhs_next) {
        // time-step mode: whole levels on one GPU with the split launches only
        // (the caller checks xstep_supported first)
        if (g_xfast == 0 || !(A.c.dgs > 0) || A.rb >= 0 || rb - ra <= g_xtile_max_rows)
            return -3;
        MarchRegions inner, edge, unused;
        // (the time-step mode keeps the separate strips: its B wave's extra
        // stage takes the XG kernel past 256 VGPRs)
        march_regions<WPB>(n, X::W, X::H, ra, rb, X::TOP_RS, X::BOT, true, inner, unused);
        march_regions<1>(n, X::W, X::H, ra, rb, X::TOP_RS, X::BOT, true, unused, edge);
        const int pm = xsmooth_launch<WPB, K, false, true>(A, inner, A.partials, lo, hi,
                                                           A.min_rows, kNormBlocks / (2 * WPB) / 2,
                                                           s);
        const int pe = xsmooth_launch<1, K, true, true>(A, edge, A.partials + pm, lo, hi,
                                                        std::min(32, A.min_rows),
                                                        kNormBlocks / 2 / 2, s);
        return pm + pe;
    }
    // inner: WPB pairs per workgroup, one workgroup per CU, long segments;
    // edge: one pair per workgroup (4 per CU) and short segments, so that its
    // ~44 K strip-rows at N=16384 (2 boundary strips + 71-row bands) take
    // about one warm-up + 44 rows per workgroup
    MarchRegions inner, edge, unused;
    // the unguarded kernel's division assumes d > 0 (div_diag<true>)
    const bool split = g_xfast != 0 && A.c.dgs > 0;
    if (A.phase != 0 && !split) return -1;   // a split pass needs the split kernels
    if (split && rb - ra <= g_xtile_max_rows) {
        const int r = xsmooth_tiled<WPB, K>(A, ra, rb, lo, hi, s);
        if (r != -2) return r;
    }
    int top, bot;
    xmargins<K>(A, ra, rb, top, bot);
    XGeo geo{};
    const bool xg =
        split && g_xgroup != 0 && xg_regions<WPB, K>(n, ra, rb, top, bot, inner, edge, geo);
    if (!xg) {
        march_regions<WPB>(n, X::W, X::H, ra, rb, top, bot, split, inner, unused);
        march_regions<1>(n, X::W, X::H, ra, rb, top, bot, split, unused, edge);
    }
    int pm = A.partials_done;
    if (A.phase != 2)
        pm = xg ? xsmooth_launch<WPB, K, false, false, true>(A, inner, A.partials, lo, hi,
                                                             A.min_rows,
                                                             kNormBlocks / (2 * WPB) / 2, s, geo)
                : xsmooth_launch<WPB, K, false>(A, inner, A.partials, lo, hi, A.min_rows,
                                                kNormBlocks / (2 * WPB) / 2, s);
    if (A.phase == 1) return pm;
    const int pe = xsmooth_launch<1, K, true>(A, edge, A.partials + pm, lo, hi,
                                              std::min(MGX_XEDGE_ROWS, A.min_rows),
                                              kNormBlocks / 2 / 2, s, geo);
    return pm + pe;
}

int launch_xsmooth(const XArgs &A, int sweeps, hipStream_t s) {
    if (A.rb >= 0 && (A.ra & 1)) return -1;   // row blocks start at even rows
    int blocks = -1;
    // 4 strip pairs per workgroup (one workgroup of 8 waves per CU): adjacent
    // 1-KiB row pieces of four strips per load (measured: 4.05 ms vs 4.13 ms
    // with 2 pairs, N=16384)
    switch (sweeps) {
        case 2: blocks = xsmooth_inst<4, 2>(A, s); break;
        case 3: blocks = xsmooth_inst<4, 3>(A, s); break;
        default: return -1;
    }
    if (A.phase == 1) return blocks;   // the norm comes with phase 2
    if (blocks > 0)
        MGX_LAUNCH(k_norm_final, dim3(1), dim3(kFinalThreads), s, (const double *)A.partials,
                   blocks, A.norm_out, A.norm_accumulate ? 2 : A.norm_sqrt ? 1 : 0);
    if (blocks > 0 && A.rhs_next)   // the next step's initial norm
        MGX_LAUNCH(k_norm_final, dim3(1), dim3(kFinalThreads), s,
                   (const double *)(A.partials + kNormBlocks), blocks, A.norm2_out, 1);
    return blocks;
}

bool xstep_supported(long n) {
    return g_xfast != 0 && n + 1 > g_xtile_max_rows;
}

long g_tile_max_n = -1;   // levels with n <= this use k_smooth_tile

void set_tile_max_n(long v) { g_tile_max_n = v; }
long get_tile_max_n();

static long tile_max_n() {
    if (g_tile_max_n < 0) {
        const char *e = getenv("MGX_TILE_MAX_N");
        // 1024: level 3 (n = 2048) as a wave march, 0.115 -> 0.105-0.110 ms
        // per cycle at N=16384 (tools/ab_levels.py); levels 4-5 measure the
        // same either way
        g_tile_max_n = e ? atol(e) : 1024;
    }
    return g_tile_max_n;
}

long get_tile_max_n() { return tile_max_n(); }

long g_tile32_min_n = -1;   // 32-row tiles on levels n >= this (tuning key "tile32_min_n")
long g_tile_xcd = -1;       // XCD-contiguous tile order (tuning key "tile_xcd")

static long tile32_min_n() {
    if (g_tile32_min_n < 0) {
        const char *e = getenv("MGX_TILE32_MIN_N");
        g_tile32_min_n = e ? atol(e) : 2048;
    }
    return g_tile32_min_n;
}
void set_tile32_min_n(long v) { g_tile32_min_n = v; }
long get_tile32_min_n() { return tile32_min_n(); }
static long tile_xcd() {
    if (g_tile_xcd < 0) {
        const char *e = getenv("MGX_TILE_XCD");
        g_tile_xcd = e ? atol(e) : 1;
    }
    return g_tile_xcd;
}
void set_tile_xcd(long v) { g_tile_xcd = v; }
long get_tile_xcd() { return tile_xcd(); }

template <int K, int MODE, int TRV>
static int smooth_tile_rows(const SmoothArgs &A, hipStream_t s) {
    using T = TileCfg<K, MODE, TRV>;
    const long n = A.n;
    const int tiles_x = (int)((n + 1 + T::TC - 1) / T::TC);
    const int tiles_y = (int)((A.rb - A.ra + T::TR - 1) / T::TR);
    const long grid = (long)tiles_x * tiles_y;
    if ((MODE & 8) && grid > kNormBlocks) return -1;
    MGX_LAUNCH((k_smooth_tile<K, MODE, TRV>), dim3((unsigned)grid), dim3(T::THREADS), s, A.uin,
               A.uout, A.rhs, A.v1, A.v2, A.uc, A.pitchc, A.rhsc, A.partials, (int)n, A.pitch,
               tiles_x, A.c, A.ra, A.rb, A.lo, A.hi, tile_xcd() ? 1 : 0);
    return (int)grid;
}

// 16 x 64 output tiles (halo overhead 2.5x the tile); with K = 3 on levels
// n >= tile32_min_n, 32 x 64 (1.9x, more work per workgroup)
template <int K, int MODE>
static int smooth_tile_inst(const SmoothArgs &A, hipStream_t s) {
    if constexpr (K == 3)
        if (A.n >= tile32_min_n()) return smooth_tile_rows<K, MODE, 32>(A, s);
    return smooth_tile_rows<K, MODE, 16>(A, s);
}

// a row block runs as LDS tiles when its march would give the resident waves
// fewer than this many rows each (tuning key "march_tile_rows"; 16: level 2
// on 4 row blocks marches, 0.50 -> 0.46 ms for the 4 parts; level 1 on 8 row
// blocks as tiles (64, 96) costs +25-45 %)
long g_march_tile_rows = 16;
void set_march_tile_rows(long v) { g_march_tile_rows = v; }
long get_march_tile_rows() { return g_march_tile_rows; }

template <int K, int MODE>
static int smooth_block(const SmoothArgs &A, hipStream_t s) {
    // the row march needs >= ~32 rows per wave to amortise its priming rows;
    // a row block too small to give every resident wave that much (a
    // partitioned level on many GPUs) runs as LDS tiles instead
    bool tile = A.n <= tile_max_n() && !(MODE & 16);   // RHSN: march only
    if (!tile && !(MODE & 16)) {
        constexpr int W4 = WCfg<K, MODE>::W * 4;
        static int slots = 0;
        if (!slots) {
            int dev = 0, cus = 0, per = 0;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_wsmooth<4, K, MODE, true>,
                                                               256, 0);
            slots = std::max(1, cus) * std::max(1, per);
        }
        const long groups = (A.n + 1 + W4 - 1) / W4;
        tile = groups * (A.rb - A.ra) < (long)slots * g_march_tile_rows;
    }
    if (tile) {
        const int g = smooth_tile_inst<K, MODE>(A, s);
        if (g > 0) return g;
    }
    // the wave-private row march (also the fallback when a tile launch would
    // need more norm partials than the buffer holds)
    return smooth_winst<4, K, MODE>(A, s);
}

template <int K>
static int smooth_k(const SmoothArgs &A, int mode, hipStream_t s) {
    switch (mode) {
        case 0: return smooth_block<K, 0>(A, s);
        case 1: return smooth_block<K, 1>(A, s);
        case 2: return smooth_block<K, 2>(A, s);
        case 4: return smooth_block<K, 4>(A, s);
        case 5: return smooth_block<K, 5>(A, s);
        case 8: return smooth_block<K, 8>(A, s);
        case 9: return smooth_block<K, 9>(A, s);
        case 10: return smooth_block<K, 10>(A, s);
        case 20: return smooth_block<K, 20>(A, s);
        default: return -1;
    }
}

int launch_smooth(const SmoothArgs &A0, int sweeps, int mode, hipStream_t s) {
    SmoothArgs A = A0;
    if (A.rb < 0) {
        A.ra = 0;
        A.rb = (int)A.n + 1;
        A.lo = 0;
        A.hi = (int)A.n;
    }
    if (A.ra & 1) return -1;   // partitions start at even rows (parity, restriction)
    int blocks = -1;
    switch (sweeps) {
        case 1: blocks = smooth_k<1>(A, mode, s); break;
        case 2: blocks = smooth_k<2>(A, mode, s); break;
        case 3: blocks = smooth_k<3>(A, mode, s); break;
        default: return -1;
    }
    if (blocks > 0 && (mode & (8 | 16)))
        MGX_LAUNCH(k_norm_final, dim3(1), dim3(kFinalThreads), s, (const double *)A.partials,
                   blocks, A.norm_out, A.norm_accumulate ? 2 : A.norm_sqrt ? 1 : 0);
    return blocks;
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
                         double *stats, hipStream_t s) {
    if (n <= kCoarseLdsMaxN && g_coarse_lds) {
        MGX_LAUNCH(k_coarse_solve_lds, dim3(1), dim3(1024), s, u, rhs, v1, v2, (int)n, pitch, c,
                   tol, maxit, zero_first ? 1 : 0, stats);
        return;
    }
    MGX_LAUNCH(k_coarse_solve, dim3(1), dim3(1024), s, u, rhs, v1, v2, (int)n, pitch, c, tol,
               maxit, zero_first ? 1 : 0, stats);
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
