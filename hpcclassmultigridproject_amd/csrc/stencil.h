// stencil.h -- internal: device-side building blocks shared by the CDNA4 stencil
// kernels (kernels.hip, wsmooth.hip, xsmooth.hip): the reference's point
// expressions, the fp_mode fma forms, row loads / stores, wave reductions,
// DPP lane shifts and the row-march work plan.  Not part of the public ABI.
#pragma once
#include "kernels.h"

#include <algorithm>
#include <cmath>

namespace mgx {

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
// two consecutive doubles from an address that is only 8-B aligned (one
// 16-B global load: the coarsest solve's column pairs start at odd columns)
__device__ __forceinline__ double2 ldu2(const double *p) {
    typedef double d2a8 __attribute__((ext_vector_type(2), aligned(8)));
    const d2a8 v = *reinterpret_cast<const d2a8 *>(p);
    return make_double2(v.x, v.y);
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

// Levels 1 and 2 of the reference tower (multigrid.cpp:148-160)
// are re-reads of the finest rank-1 velocity through the injection's index
// quirk: with s = 2^(l-1), W = N/4 + 1, level l's entry (i, j) is the finest
// entry (I, c) = (2s i + q, 2s j - q(2W-1)) with q = floor(s(j-i)/W), where s(i(2W-1) + j) < W^2, and zero beyond (the
// injection's zero fill).  So v1(i, j) = fl(sa1[I] * sb1[c]) bit for bit
// wherever the finest field is its exact factors (checked entry by entry at
// upload, launch_vgen_check).  For a fixed column j, as the march goes down
// the rows, q takes at most two values (the nonzero rows, i < ~W/(2s), move
// s(j-i) by less than W): state 0 (q = qh = floor(s j/W)) for i < rt, state
// 1 (q = qh - 1) for rt <= i < rz, state 2 (zero) for i >= rz.  (VGen:
// kernels.h; tests/test_vgen_formula.py checks the closed form against the
// CPU checker's tower.)
//
// strided (MGX_TOWER_CORRECT, any level l >= 1): each level is the injection
// of the one above, so entry (i, j) is the finest entry (2^l i, 2^l j) and
// v1(i, j) = fl(sa1[2^l i] * sb1[2^l j]) -- one state (q = 0) on every row.
struct VGCol {
    int qh, rt, rz, chi, clo;   // chi / clo: the finest column of states 0 / 1
};
__host__ __device__ inline VGCol vg_col(int j, int n, int l, bool strided = false) {
    VGCol k;
    if (j < 0 || j > n) {   // outside the level: every row zero
        k.qh = 0;
        k.rt = 0;
        k.rz = -0x7fffffff;
        k.chi = k.clo = 0;
        return k;
    }
    if (strided) {
        k.qh = 0;
        k.rt = k.rz = 0x7fffffff;
        k.chi = k.clo = j << l;
        return k;
    }
    const int N = n << l, W = N / 4 + 1, den = 2 * W - 1, s = 1 << (l - 1);
    k.qh = s * j / W;
    k.rt = (s * j - k.qh * W) / s + 1;
    k.rz = (W * W - s * j + s * den - 1) / (s * den);
    const int chi = 2 * s * j - k.qh * den, clo = chi + den;
    k.chi = chi < 0 ? 0 : (chi > N ? N : chi);   // (an unused state's column: any valid)
    k.clo = clo < 0 ? 0 : (clo > N ? N : clo);
    return k;
}
__host__ __device__ inline int vg_state(const VGCol &k, int i) {
    return i >= k.rz ? 2 : (i >= k.rt ? 1 : 0);
}
// the finest row I of state st (N+1: the zero entry of VGen::a)
__host__ __device__ inline int vg_row(const VGCol &k, int i, int st, int l, int N) {
    return st == 2 ? N + 1 : (i << l) + k.qh - st;
}

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

// ---------------------------------------------------------------- fp_mode fma
// MGX_FP_FMA (Coef::fm): the smoothing passes evaluate gs.cpp:126-130 divided
// by the diagonal d and contracted,
//   u = f' + mn*uN + mw*uW + me*uE + ms*uS,   f' = f/d,  m = -(coefficient)/d,
// with t = v*h/2, g = rr/d, gn = g*nu:
//   mn = g*t1 - gn, mw = g*t2 - gn   (-cc/d from v1, -aa/d from v2), one fma;
//   ms = c2 - mn,   me = c2 - mw     (-dd/d, -bb/d: cc + dd = aa + bb = 2 rr nu,
//                                     c2 = -2 gn), one subtraction --
// four v_fma_f64 per update against 4 mul + 4 sub + the 3-op division of the
// bitwise form (gs.cpp:130 evaluated term by term).  The residual (gs.cpp:75)
// is d*(GS update - u).  Not bitwise the reference: each value within a few
// ulp (max|duT| <= 1e-12, the same cycle counts).  The freshest
// neighbour (uS, written by the previous stage of the same step) enters last.
// Every kernel (row marches, LDS tiles, coarsest solve) forms the same values
// from t = fl(v*h/2) with the same operations -- a kernel may keep ms / me per
// row or recompute them per update (fewer registers), the bits are the same --
// so fma-mode results do not depend on which kernel, tile size or row
// partition computed a point.
__device__ __forceinline__ double fm_mp(double t, const Coef &c) {   // mn / mw
    return __builtin_fma(c.g, t, -c.gn);
}
__device__ __forceinline__ double fm_ms(double m, const Coef &c) {   // ms / me from mn / mw
    return c.c2 - m;
}
__device__ __forceinline__ double fm_upd(double fs, double mn, double uN, double mw, double uW,
                                         double ms, double uS, double me, double uE) {
    return __builtin_fma(ms, uS,
                         __builtin_fma(me, uE, __builtin_fma(mw, uW, __builtin_fma(mn, uN, fs))));
}
__device__ __forceinline__ double fm_res(double fs, double u, double mn, double uN, double mw,
                                         double uW, double ms, double uS, double me, double uE,
                                         const Coef &c) {
    return (fm_upd(fs, mn, uN, mw, uW, ms, uS, me, uE) - u) * c.dgs;
}
// from mn, mw only (ms, me recomputed)
__device__ __forceinline__ double fm_upd2(double fs, double mn, double uN, double mw, double uW,
                                          double uS, double uE, const Coef &c) {
    return fm_upd(fs, mn, uN, mw, uW, fm_ms(mn, c), uS, fm_ms(mw, c), uE);
}
__device__ __forceinline__ double fm_res2(double fs, double u, double mn, double uN, double mw,
                                          double uW, double uS, double uE, const Coef &c) {
    return fm_res(fs, u, mn, uN, mw, uW, fm_ms(mn, c), uS, fm_ms(mw, c), uE, c);
}
// from t1, t2 (no stored coefficients)
__device__ __forceinline__ double fm_upd_t(double fs, double t1, double t2, double uN, double uW,
                                           double uS, double uE, const Coef &c) {
    return fm_upd2(fs, fm_mp(t1, c), uN, fm_mp(t2, c), uW, uS, uE, c);
}
__device__ __forceinline__ double fm_res_t(double fs, double t1, double t2, double u, double uN,
                                           double uW, double uS, double uE, const Coef &c) {
    return fm_res2(fs, u, fm_mp(t1, c), uN, fm_mp(t2, c), uW, uS, uE, c);
}

inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }

#define MGX_LAUNCH(kern, grid, block, s, ...) \
    hipLaunchKernelGGL((kern), (grid), (block), 0, (s), __VA_ARGS__)

// k_norm_final over `count` partials (kernels.hip): mode 1 = *out = sqrt of the
// sum, 0 = the sum, 2 = *out += the sum
void launch_norm_final(const double *partials, int count, double *out, int mode,
                       hipStream_t s);

template <int WPB>
inline void add_region(MarchRegions &r, int sfirst, int slim, int r0, int r1) {
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
inline void march_split(long n, int W, int H, int ra, int rb, int top, int bot, int &si0,
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
inline void march_regions(long n, int W, int H, int ra, int rb, int top, int bot, bool split,
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

// Row-march work plan (kernels.hip): knobs march_order / march_seg /
// march_min_rows, the ordered regions and the workgroup count of a launch.
MarchRegions order_regions(const MarchRegions &reg, long upw);
unsigned plan_march(const MarchRegions &reg, int wpb, long slots, long min_rows, long max_wgs,
                    int warm, long &upw, MarchRegions &out);


// ------------------------------------------------------- coarsest solve in LDS
// The coarsest solve (k_coarse_solve, kernels.hip) with u held in LDS and each thread's rhs / v1 / v2 (FM: f',
// t1, t2) in registers (n <= 64): the loop touches no global memory.  Same
// sweep order, term order and reduction order as k_coarse_solve, so u, the
// norms and the iteration count are bitwise those of k_coarse_solve.
//
// Latency and LDS issue, not work, are the cost of this kernel (~4 K points):
//   * the 1024 threads map onto the interior as (row 1 + (t >> 5) + 32p,
//     columns 2(t & 31) + 1 and + 2): four points per thread, two of each
//     colour, every lane busy; a colour stage first reads the neighbours of
//     its two points, then stores both updates (the points of a colour are
//     independent);
//   * the set-up loads each row's column pair of rhs / v1 / v2 as ONE 16-B
//     load (6 per thread instead of 24 scalar loads of the earlier layout,
//     whose separate residual points needed their own copies), all in flight
//     at once from clamped addresses, masks applied after;
//   * the residual runs on the same four points from the same registers and
//     is summed in a fixed order (p, then colour; then the wave butterfly,
//     then the 16 wave partials in order, by EVERY thread, so the norm needs
//     no broadcast barrier): three barriers per iteration (two colour stages,
//     the partials) instead of five;
//   * every loop is unrolled to its fixed trip count for n <= 64, guarded.
// reps: the solve repeated back to back (a W-cycle visits the coarsest level
// `shape` times in a row, multigrid.cpp:52-65) in this one launch.
//
// As a device function for one workgroup of 1024 threads: k_coarse_solve_lds
// (kernels.hip) is this alone; k_smooth_tile (wsmooth.hip, CoarseFuse) runs it
// first in every workgroup of the pass above the coarsest level and prolongs
// from the LDS copy (write = false in all but one workgroup, which stores u
// and the iteration statistics as the kernel does).  su: kCoarseLdsNP^2
// doubles of LDS, lds: 16, s_norm: unused (kept for the callers' layout).
// (kCoarseLdsMaxN, kCoarseLdsNP: kernels.h)
template <bool FM>
__device__ __forceinline__ void coarse_lds_body(double *su, double *lds, double *s_norm, double *u,
                                                const double *rhs, const double *v1,
                                                const double *v2, int n, long pitch, Coef c,
                                                double tol, int maxit, int zero_first, int reps,
                                                double *stats, bool write) {
    (void)s_norm;
    constexpr int NP = kCoarseLdsNP;
    constexpr int GP = kCoarseLdsMaxN / 32;   // rows per thread: 1 + gr + 32p
    const int t = threadIdx.x;
    const int tx = t & 63, ty = t >> 6;
    const int gk = t & 31, gr = t >> 5;
    const double hh = c.h * 0.5;
    // per-point constants in registers: (f, t1, t2) = FM ? (rhs/d, v1*h/2, v2*h/2)
    // : (rhs, v1, v2), exactly the operands the L2 version reads per use.
    // Colour c of row i sits at column 1 + ((i + 1 + c) & 1) + 2 gk: the pair
    // (2gk + 1, 2gk + 2) holds both colours, colour 0 first on odd rows.
    {   // u into LDS first (its loads and registers are done before the
        // colour points' set-up): rows ty + 16m (m <= 4), columns tx, tx + 64
        constexpr int MF = (kCoarseLdsMaxN + 16) / 16;
        double a[MF][2] = {};
        if (!zero_first)   // (clamped addresses: every load in flight at once)
#pragma unroll
            for (int m = 0; m < MF; ++m)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    a[m][h] = u[(long)min(ty + 16 * m, n) * pitch + min(tx + 64 * h, n)];
#pragma unroll
        for (int m = 0; m < MF; ++m)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = ty + 16 * m, j = tx + 64 * h;
                if (i <= n && j <= n) su[i * NP + j] = zero_first ? 0.0 : a[m][h];
            }
    }
    double gf[2][GP], gx[2][GP], gy[2][GP];
    int gq[2][GP];
    bool gon[2][GP];
    const bool odd = !(gr & 1);   // row 1 + gr + 32p is odd
    {
        double2 lr[GP], lx[GP], ly[GP];
#pragma unroll
        for (int p = 0; p < GP; ++p) {   // every load in flight before any use
            const int i = 1 + gr + 32 * p;
            const bool ok = i <= n - 1 && 2 * gk + 2 <= n;
            const long q = ok ? (long)i * pitch + 2 * gk + 1 : pitch + 1;
            lr[p] = ldu2(rhs + q);
            lx[p] = ldu2(v1 + q);
            ly[p] = ldu2(v2 + q);
        }
#pragma unroll
        for (int p = 0; p < GP; ++p) {
            const int i = 1 + gr + 32 * p;
#pragma unroll
            for (int colour = 0; colour < 2; ++colour) {
                const bool lo = (colour == 0) == odd;   // column 2gk + 1
                const int j = lo ? 2 * gk + 1 : 2 * gk + 2;
                const bool on = i <= n - 1 && j <= n - 1;
                gon[colour][p] = on;
                gq[colour][p] = on ? i * NP + j : NP + 1;
                const double f = lo ? lr[p].x : lr[p].y, x = lo ? lx[p].x : lx[p].y,
                             y = lo ? ly[p].x : ly[p].y;
                gf[colour][p] = on ? (FM ? f * c.rdgs : f) : 0.0;
                gx[colour][p] = on ? (FM ? x * hh : x) : 0.0;
                gy[colour][p] = on ? (FM ? y * hh : y) : 0.0;
            }
        }
    }
    if (write && zero_first)   // (the row padding, as the L2 version leaves it)
        for (int i = ty; i <= n; i += 16)
            for (int j = n + 1 + tx; j < pitch; j += 64) u[(long)i * pitch + j] = 0.0;
    __syncthreads();
    int total = 0;
    double res = 1.0;
    for (int rep = 0; rep < reps; ++rep) {
        int it = 0;
        res = 1.0;
        while (it < maxit && res > tol) {
#pragma unroll
            for (int colour = 0; colour < 2; ++colour) {
                double nN[GP], nW[GP], nS[GP], nE[GP];
#pragma unroll
                for (int p = 0; p < GP; ++p) {
                    const int q = gq[colour][p];
                    nN[p] = su[q - NP];
                    nW[p] = su[q - 1];
                    nS[p] = su[q + NP];
                    nE[p] = su[q + 1];
                }
#pragma unroll
                for (int p = 0; p < GP; ++p) {
                    if (!gon[colour][p]) continue;
                    su[gq[colour][p]] =
                        FM ? fm_upd_t(gf[colour][p], gx[colour][p], gy[colour][p], nN[p], nW[p],
                                      nS[p], nE[p], c)
                           : gs_point(gf[colour][p], gx[colour][p], gy[colour][p], nN[p], nW[p],
                                      nS[p], nE[p], c);
                }
                __syncthreads();
            }
            double acc = 0.0;
#pragma unroll
            for (int p = 0; p < GP; ++p) {
                double rr[2];
#pragma unroll
                for (int colour = 0; colour < 2; ++colour) {
                    const int q = gq[colour][p];
                    const double f = gf[colour][p], x = gx[colour][p], y = gy[colour][p];
                    rr[colour] = FM ? fm_res_t(f, x, y, su[q], su[q - NP], su[q - 1],
                                               su[q + NP], su[q + 1], c)
                                    : res_point(f, x, y, su[q], su[q - NP], su[q - 1],
                                                su[q + NP], su[q + 1], c);
                }
#pragma unroll
                for (int colour = 0; colour < 2; ++colour)
                    if (gon[colour][p]) acc += rr[colour] * rr[colour];
                // (one row's LDS reads at a time: the workgroup's 1024 threads
                // leave 128 VGPRs, and all four points' reads at once spilled
                // in the fused tile kernels)
                __builtin_amdgcn_sched_barrier(0);
            }
            // the block sum in every thread: wave butterfly, then the 16 wave
            // partials in order -- the same bits everywhere, no broadcast
            // (the next write of lds[] is behind the next iteration's two
            // colour barriers, so no thread can overwrite what another reads)
            acc = wave_sum(acc);
            if ((t & 63) == 0) lds[t >> 6] = acc;
            __syncthreads();
            double s = 0.0;
#pragma unroll
            for (int w = 0; w < 16; ++w) s += lds[w];
            res = sqrt(s);
            ++it;
        }
        total += it;
    }
    if (!write) return;
    for (int i = ty; i <= n; i += 16)
        for (int j = tx; j <= n; j += 64) u[(long)i * pitch + j] = su[i * NP + j];
    if (t == 0) {
        stats[0] += total;
        stats[1] = res;
    }
}

}  // namespace mgx
