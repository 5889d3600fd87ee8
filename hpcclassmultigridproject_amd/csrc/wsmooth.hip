// wsmooth.hip -- the fused K-sweep smoothing pass of one level (levels below
// the finest, and the finest level's first pre-smoothing of a run): the
// wave-private row march (k_wsmooth) for large levels, 2-D LDS tiles
// (k_smooth_tile) for small ones, and launch_smooth.
#include "stencil.h"

#include <type_traits>

namespace mgx {
namespace {

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
#ifndef MGX_WMINB
#define MGX_WMINB 1
#endif
    // workgroups per CU the compiler must fit (launch bounds)
    static constexpr int MINB = MGX_WMINB;
};

// rhs/v prefetch distance of the wave march: with t = v*h/2 formed at the
// row's first use (scale_rv), 4 steps measured -3 % on level 1 against 2
// (3: -2 %, 5: -2 %; tools/ab_libs.sh)
#ifndef MGX_WRV
#define MGX_WRV 4
#endif
#ifndef MGX_WU
#define MGX_WU 2
#endif


// G = false: the unguarded march (interior strips, rows [TOP, n+1-BOT) of
// WCfg: no per-stage predicates), G = true: guarded (see k_xsmooth).
// PD: the diagonal is positive (every nu <= 0): the shorter division (div_diag).
// Each row's x-neighbour coefficient pair (cn, cs, from t1) is formed once, at
// the row's first stage, the y pair (from t2) in every stage: all four per row
// (as in k_xsmooth) needs ~110 more VGPRs -- one wave per SIMD, measured
// slower.  (RHSN: every coefficient per stage.)
// FM: fp_mode fma (stencil.h): f' = f/d enters the ring at the row's first
// use, the stored pair is mn, mw (ms, me recomputed: one subtraction each),
// the stages contract (four fmas), residuals
// are d*(update - u); RHSN's rhs keeps the reference expressions (gs.cpp:44,
// stored unscaled) and is scaled after.
// VG: levels 1-2 of the reference tower, or every level of the correct tower
// (vg.strided), v1 / v2 generated from the finest
// factors (stencil.h vg_col): per row two cached loads of the (sa1, sa2) pairs
// of the lane's two columns replace the two HBM row loads; the lane's sb pairs
// (three states per column) sit in its LDS slice and are multiplied in at the
// row's first use -- the same operands as the tower's entries, bitwise.
template <int WPB, int K, int MODE, bool G, bool PD = false, bool FM = false, bool VG = false>
__global__ __launch_bounds__(64 * WPB, (WCfg<K, MODE>::MINB)) void k_wsmooth(
    const double *__restrict__ uin, double *__restrict__ uout, const double *__restrict__ rhs,
    const double *__restrict__ v1, const double *__restrict__ v2, const double *__restrict__ uc,
    long pitchc, double *__restrict__ rhsc, double *__restrict__ partials, int n, long pitch,
    MarchRegions reg, long units_per_wg, Coef c, int lo, int hi, double *__restrict__ rhs_out,
    const double *__restrict__ zrow, int vz, VGen vg) {
    using C = WCfg<K, MODE>;
    __shared__ double2 vgl[VG ? 64 * WPB * 6 : 1];
    constexpr int S = C::S, E = C::E, H = C::H, NR = C::NR, W = C::W;
    // rhs/v prefetch distance in steps (row s+WRV takes the slot of row
    // s+WRV-NR, last used by the residual stage on row s+1-S); RHSN uses a
    // row's v two steps before its first stage
    constexpr int WRV = C::RHSN ? (MGX_WRV > 4 ? MGX_WRV : 4) : MGX_WRV;
    static_assert(WRV >= 2 && WRV <= NR - S + 1, "rhs/v prefetch distance");
    // u rows (+ coarse parents) WU steps ahead of entering the u ring
    constexpr int WU = MGX_WU < NR - 3 ? MGX_WU : NR - 3;
    static_assert(WU >= 1 && WU <= NR - 3, "u prefetch distance");
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
        VGCol g0{}, g1{};
        // slot k of lane t at vgl[k * NT + t] (slot-major: the lanes of a
        // wave read consecutive 16-B words; lane-major, stride 96 B, was an
        // 8-way LDS bank conflict on every read -- 5 M conflict cycles per
        // level-1 pass in the round-4 PMC profile)
        constexpr int NT = 64 * WPB;
        const int lb = threadIdx.x;
        if constexpr (VG) {   // (lane-private slice: no barrier)
            g0 = vg_col(c0, n, vg.l, vg.strided);
            g1 = vg_col(c0 + 1, n, vg.l, vg.strided);
            vgl[lb + 0 * NT] = make_double2(vg.b1[g0.chi], vg.b2[g0.chi]);
            vgl[lb + 1 * NT] = make_double2(vg.b1[g0.clo], vg.b2[g0.clo]);
            vgl[lb + 2 * NT] = make_double2(0.0, 0.0);
            vgl[lb + 3 * NT] = make_double2(vg.b1[g1.chi], vg.b2[g1.chi]);
            vgl[lb + 4 * NT] = make_double2(vg.b1[g1.clo], vg.b2[g1.clo]);
            vgl[lb + 5 * NT] = make_double2(0.0, 0.0);
        }

        struct UPre {
            double2 X;
            double q00, q01, q10, q11;
        };
        // u rows (+ coarse parents) in flight, a ring by row like rd: row R in
        // slot R mod NR, loaded WU steps before it enters the u ring
        UPre up[NR];
#pragma unroll
        for (int q = 0; q < NR; ++q) up[q] = UPre{make_double2(0.0, 0.0), 0.0, 0.0, 0.0, 0.0};
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
                if (odd) {   // (a row clamped to an even one: its own parent)
                    const int o1 = (Rc & 1) ? ipc : 0;
                    u.q10 = p0[o1];
                    u.q11 = p0[o1 + j1];
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
            if constexpr (VG) {   // (sa1, sa2) of column c0 in x, c0+1 in y
                d.x = vg.a[vg_row(g0, Rc, vg_state(g0, Rc), vg.l, n << vg.l)];
                d.y = vg.a[vg_row(g1, Rc, vg_state(g1, Rc), vg.l, n << vg.l)];
                return;
            }
            const bool z = Rc >= vz;
            d.x = ld2((z ? zrow : v1 + o) + cl);
            d.y = ld2((z ? zrow : v2 + o) + cl);
        };
        // (FM: and f' = f/d; RHSN forms the rhs after this, see rhs_norm)
        auto scale_rv = [&](RowData &d, const int R) {
            if constexpr (VG) {   // v = fl(a * b) of row R's states
                const int Rc = min(max(R, lo), hi);
                const double2 b0 = vgl[lb + vg_state(g0, Rc) * NT];
                const double2 b1 = vgl[lb + (3 + vg_state(g1, Rc)) * NT];
                const double2 a0 = d.x, a1 = d.y;
                d.x = make_double2(a0.x * b0.x, a1.x * b1.x);
                d.y = make_double2(a0.y * b0.y, a1.y * b1.y);
            }
            d.x = make_double2(d.x.x * hh, d.x.y * hh);
            d.y = make_double2(d.y.x * hh, d.y.y * hh);
            if (FM && !C::RHSN) d.r = make_double2(d.r.x * c.rdgs, d.r.y * c.rdgs);
        };

        const int s_first = a - E;
        const int s_last = b + E - 3;
        int s = s_first >= 0 ? (s_first / NR) * NR : -(((-s_first) + NR - 1) / NR) * NR;
        s = __builtin_amdgcn_readfirstlane(s);

        double2 ur[NR];
        RowData rd[NR];
#ifndef MGX_WH
#define MGX_WH 1
#endif
        constexpr bool WH = MGX_WH && !C::RHSN;   // cn, cs stored per row
        CoefRow cf[NR];
#pragma unroll
        for (int q = 0; q < NR; ++q) {
            ur[q] = make_double2(0.0, 0.0);
            rd[q].r = rd[q].x = rd[q].y = make_double2(0.0, 0.0);
            const double2 z = make_double2(0.0, 0.0);
            cf[q] = CoefRow{z, z, z, z};
        }
        // residual (gs.cpp:75 term order) of the row in slot iR, column c0 / c0+1,
        // from its stored cn, cs (FM: mn, ms)
        auto res_cx = [&](const int iR, const int iN, const int iS, const double uW) {
            const CoefRow &k = cf[iR];
            if (FM)   // (stored: mn in cn, mw in cw)
                return fm_res2(rd[iR].r.x, ur[iR].x, k.cn.x, ur[iN].x, k.cw.x, uW, ur[iS].x,
                               ur[iR].y, c);
            const double t2 = rd[iR].y.x;
            const double cw = c.rr * (c.nu - t2), ce = c.rr * (t2 + c.nu);
            return rd[iR].r.x - (c.dgs * ur[iR].x + k.cn.x * ur[iN].x + cw * uW +
                                 k.cs.x * ur[iS].x + ce * ur[iR].y);
        };
        auto res_cy = [&](const int iR, const int iN, const int iS, const double uE) {
            const CoefRow &k = cf[iR];
            if (FM)
                return fm_res2(rd[iR].r.y, ur[iR].y, k.cn.y, ur[iN].y, k.cw.y, ur[iR].x,
                               ur[iS].y, uE, c);
            const double t2 = rd[iR].y.y;
            const double cw = c.rr * (c.nu - t2), ce = c.rr * (t2 + c.nu);
            return rd[iR].r.y - (c.dgs * ur[iR].y + k.cn.y * ur[iN].y + cw * ur[iR].x +
                                 k.cs.y * ur[iS].y + ce * uE);
        };
        // prologue (s == 0 mod NR): u rows s..s+2 in the ring, s+3 / s+4 in
        // flight (sets 1 / 0), rhs/v rows s+1, s+2 loaded
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            load_u(s + d, up[d], d & 1);
            ur[d] = make_u(s + d, up[d], d & 1);
        }
#pragma unroll
        for (int d = 3; d < 3 + WU; ++d) load_u(s + d, up[d % NR], d & 1);
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
            d.r = FM ? make_double2(f0 * c.rdgs, f1 * c.rdgs) : make_double2(f0, f1);
            if (rowin(r) && r >= 1 && r <= n - 1 && keep) {
                double *row = rhs_out + rowoff(r, ip);
                if (in0 && in1) {
                    st2(row + c0, make_double2(f0, f1));
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
            scale_rv(rd[1], s + 1);
            rhs_norm(s + 1, 1, 0, 2);   // the first stage's row
        }

        for (;;) {
#pragma unroll
            for (int p = 0; p < NR; ++p) {
                // (1) u row s+3 enters the ring; its prefetch set takes row s+5
                ur[(p + 3) % NR] = make_u(s + 3, up[(p + 3) % NR], (p + 3) & 1);
                load_u(s + 3 + WU, up[(p + 3 + WU) % NR], (p + 3 + WU) & 1);
                // t of the row first used in this step: s+2 (RHSN), else s+1
                scale_rv(rd[(p + (C::RHSN ? 2 : 1)) % NR], s + (C::RHSN ? 2 : 1));
                if (WH) {   // cn, cs of row s+1 from t1 (gs.cpp:128-129's cc, dd)
                    const RowData &d1 = rd[(p + 1) % NR];
                    CoefRow &k1 = cf[(p + 1) % NR];
                    if (FM) {   // mn, mw (ms, me recomputed per stage: 8 VGPRs per row fewer)
                        k1.cn = make_double2(fm_mp(d1.x.x, c), fm_mp(d1.x.y, c));
                        k1.cw = make_double2(fm_mp(d1.y.x, c), fm_mp(d1.y.y, c));
                    } else {
                        k1.cn = make_double2(c.rr * (c.nu - d1.x.x), c.rr * (c.nu - d1.x.y));
                        k1.cs = make_double2(c.rr * (d1.x.x + c.nu), c.rr * (d1.x.y + c.nu));
                    }
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
                            if (FM && WH)
                                ur[iR].x = fm_upd2(d.r.x, k.cn.x, ur[iN].x, k.cw.x, uW, ur[iS].x,
                                                   ur[iR].y, cg);
                            else if (FM)
                                ur[iR].x = fm_upd_t(d.r.x, d.x.x, d.y.x, ur[iN].x, uW, ur[iS].x,
                                                    ur[iR].y, cg);
                            else if (WH)
                                ur[iR].x = div_diag<PD>(d.r.x - k.cn.x * ur[iN].x -
                                                            cg.rr * (cg.nu - d.y.x) * uW -
                                                            k.cs.x * ur[iS].x -
                                                            cg.rr * (d.y.x + cg.nu) * ur[iR].y,
                                                        c);
                            else
                                ur[iR].x = gs_point_t<PD>(d.r.x, d.x.x, d.y.x, ur[iN].x, uW,
                                                          ur[iS].x, ur[iR].y, cg);
                        }
                    } else {
                        const double uE = dpp_shl1(ur[iR].x);   // column c0+2
                        if (!G || (inr && in1)) {
                            if (FM && WH)
                                ur[iR].y = fm_upd2(d.r.y, k.cn.y, ur[iN].y, k.cw.y, ur[iR].x,
                                                   ur[iS].y, uE, cg);
                            else if (FM)
                                ur[iR].y = fm_upd_t(d.r.y, d.x.y, d.y.y, ur[iN].y, ur[iR].x,
                                                    ur[iS].y, uE, cg);
                            else if (WH)
                                ur[iR].y = div_diag<PD>(d.r.y - k.cn.y * ur[iN].y -
                                                            cg.rr * (cg.nu - d.y.y) * ur[iR].x -
                                                            k.cs.y * ur[iS].y -
                                                            cg.rr * (d.y.y + cg.nu) * uE,
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
                        if (WH) return res_cx(iR, iN, iS, uW);
                        if (FM)
                            return fm_res_t(d.r.x, d.x.x, d.y.x, ur[iR].x, ur[iN].x, uW, ur[iS].x,
                                            ur[iR].y, c);
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
                            if (WH) return res_cy(iR, iN, iS, uE);
                            if (FM)
                                return fm_res_t(d.r.y, d.x.y, d.y.y, ur[iR].y, ur[iN].y, ur[iR].x,
                                                ur[iS].y, uE, c);
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

// FM: fp_mode fma (stencil.h): f' = f/d and t = v*h/2 kept per pair, the
// contracted update and residual from them.
template <int K, int MODE, int TRV, bool FM>
__global__ __launch_bounds__(MGX_TILE_THREADS) void k_smooth_tile(
    const double *__restrict__ uin, double *__restrict__ uout, const double *__restrict__ rhs,
    const double *__restrict__ v1, const double *__restrict__ v2, const double *__restrict__ uc,
    long pitchc, double *__restrict__ rhsc, double *__restrict__ partials, int n, long pitch,
    int tiles_x, Coef c, int ra, int rb, int lo, int hi, int xcd, CoarseFuse cf) {
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

    // cf.on (prolongation passes): the coarse level is solved here first, in
    // LDS, by every workgroup alike (the same operations: the same bits), and
    // the prolongation reads that copy; workgroup 0 stores it (CoarseFuse)
    __shared__ double csu[C::PROL ? kCoarseLdsNP * kCoarseLdsNP : 1];
    __shared__ double cred[C::PROL ? 16 : 1];
    __shared__ double cnorm;
    if constexpr (C::PROL) {
        // (its thread layout, trip counts and 16 reduction slots are fixed)
        static_assert(T::THREADS == 1024, "coarse_lds_body needs 1024 threads per workgroup");
        if (cf.on)
            coarse_lds_body<FM>(csu, cred, &cnorm, cf.u, cf.rhs, cf.v1, cf.v2, (int)cf.n,
                                cf.pitch, cf.c, cf.tol, cf.maxit, cf.zero_first, cf.reps,
                                cf.stats, blockIdx.x == 0);
    }
    // coarse u (i, j): the LDS copy or HBM
    auto cu = [&](long i, long j) {
        return (C::PROL && cf.on) ? csu[i * kCoarseLdsNP + j] : uc[i * pitchc + j];
    };

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
                const double q00 = cu(ii, jj), q01 = (jj + 1 <= nc) ? cu(ii, jj + 1) : 0.0;
                double2 pr;
                if (!(gi & 1)) {
                    pr.x = q00;
                    pr.y = (q00 + q01) / 2;
                } else {
                    const double q10 = cu(ii + 1, jj),
                                 q11 = (jj + 1 <= nc) ? cu(ii + 1, jj + 1) : 0.0;
                    pr.x = (q00 + q10) / 2;
                    pr.y = (q00 + q10 + q01 + q11) / 4;
                }
                v.x = v.x + pr.x;
                v.y = v.y + pr.y;
            }
            const double2 rr = ld2(rhs + o), xx = ld2(v1 + o), yy = ld2(v2 + o);
            f0[m] = FM ? rr.x * c.rdgs : rr.x;
            f1[m] = FM ? rr.y * c.rdgs : rr.y;
            const double hh = FM ? c.h * 0.5 : 1.0;   // (an exact no-op scaling otherwise)
            x0[m] = FM ? xx.x * hh : xx.x;
            x1[m] = FM ? xx.y * hh : xx.y;
            y0[m] = FM ? yy.x * hh : yy.x;
            y1[m] = FM ? yy.y * hh : yy.y;
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
            own[b] = FM ? fm_upd_t(fr, fx, fy, oth[b - HW], oth[b - 1 + cs], oth[b + HW],
                                   oth[b + cs], c)
                        : gs_point_fast(fr, fx, fy, oth[b - HW], oth[b - 1 + cs], oth[b + HW],
                                        oth[b + cs], c);
        }
        __syncthreads();
    }

    double acc = 0.0;
    // gs.cpp:75 (FM: d*(update - u))
    auto tres = [&](double f, double x, double y, double u, double uN, double uW, double uS,
                    double uE, const Coef &cc) {
        return FM ? fm_res_t(f, x, y, u, uN, uW, uS, uE, cc)
                  : res_point(f, x, y, u, uN, uW, uS, uE, cc);
    };
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
                        tres(f0[m], x0[m], y0[m], p0[b], p1[b - HW], p1[b - 1], p1[b + HW],
                                  p1[b], c);
            } else {
                if (in0) {
                    const double res = tres(f0[m], x0[m], y0[m], p0[b], p1[b - HW],
                                                 p1[b - 1], p1[b + HW], p1[b], c);
                    acc += res * res;
                }
                if (in1) {
                    const double res = tres(f1[m], x1[m], y1[m], p1[b], p0[b - HW],
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

}  // namespace

template <int WPB, int K, int MODE, bool G, bool PD, bool FM, bool VG>
static int wsmooth_launch_pd(const SmoothArgs &A, const MarchRegions &reg, double *partials,
                             long max_wgs, hipStream_t s) {
    const long total = reg.pre[reg.count];
    if (total <= 0) return 0;
    static int slots = 0;   // resident workgroups of this instantiation
    if (!slots) {
        int dev = 0, cus = 0, per = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_wsmooth<WPB, K, MODE, G, PD, FM, VG>,
                                                           64 * WPB, 0);
        slots = std::max(1, cus) * std::max(1, per);
    }
    long upw;
    MarchRegions r;
    // one segment per workgroup when the last band is short (warm-up ~E + NR/2
    // rows: the prologue aligns the first step to NR): level 1 at N=16384
    // 1.11 -> 1.075 ms (its 19 last-band workgroups each marched pieces of two
    // strips); the same per rank on 8 row blocks
    const unsigned grid = plan_march(reg, WPB, slots, get_march_min_rows(), max_wgs,
                                     WCfg<K, MODE>::E + WCfg<K, MODE>::NR / 2, upw, r);
    MGX_LAUNCH((k_wsmooth<WPB, K, MODE, G, PD, FM, VG>), dim3(grid), dim3(64 * WPB), s, A.uin,
               A.uout, A.rhs, A.v1, A.v2, A.uc, A.pitchc, A.rhsc, partials, (int)A.n, A.pitch, r,
               upw, A.c, A.lo, A.hi, A.rhs_out, A.zrow ? A.zrow : A.v1,
               A.zrow ? A.vz : 0x7fffffff, A.vg);
    return (int)grid * WPB;   // NORM partials written
}
// the short division when the diagonal is positive (every nu <= 0)
template <int WPB, int K, int MODE, bool G, bool VG = false>
static int wsmooth_launch(const SmoothArgs &A, const MarchRegions &reg, double *partials,
                          long max_wgs, hipStream_t s) {
    // (fp_mode fma: no division)
    if (A.c.fm)
        return wsmooth_launch_pd<WPB, K, MODE, G, false, true, VG>(A, reg, partials, max_wgs, s);
    if (A.c.dgs > 0)
        return wsmooth_launch_pd<WPB, K, MODE, G, true, false, VG>(A, reg, partials, max_wgs, s);
    return wsmooth_launch_pd<WPB, K, MODE, G, false, false, VG>(A, reg, partials, max_wgs, s);
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
    // the generated velocity: the V-cycle's 3-sweep pre / post passes (and a
    // W-cycle's second pre-smoothing of a visit, from a non-zero u)
    if constexpr (K == 3 && (MODE == (kModeZero | kModeRestrict) || MODE == kModeProlong ||
                             MODE == kModeRestrict))
        if (A.vg.a) return wsmooth_launch<WPB, K, MODE, true, true>(A, edge, A.partials,
                                                                     kNormBlocks / WPB, s);
    return wsmooth_launch<WPB, K, MODE, true>(A, edge, A.partials, kNormBlocks / WPB, s);
}

// levels with n <= tile_max_n use k_smooth_tile (tuning key "tile_max_n"):
// 1024 = level 3 (n = 2048) as a wave march, 0.115 -> 0.105-0.110 ms per
// cycle at N=16384 (tools/ab_levels.py); levels 4-5 measure the same either way
long g_tile_max_n = 1024;
void set_tile_max_n(long v) { g_tile_max_n = v; }
long get_tile_max_n() { return g_tile_max_n; }
long g_tile32_min_n = 2048;   // 32-row tiles on levels n >= this (tuning key "tile32_min_n")
void set_tile32_min_n(long v) { g_tile32_min_n = v; }
long get_tile32_min_n() { return g_tile32_min_n; }
long g_tile_xcd = 1;          // XCD-contiguous tile order (tuning key "tile_xcd")
void set_tile_xcd(long v) { g_tile_xcd = v; }
long get_tile_xcd() { return g_tile_xcd; }

template <int K, int MODE, int TRV>
static int smooth_tile_rows(const SmoothArgs &A, hipStream_t s) {
    using T = TileCfg<K, MODE, TRV>;
    const long n = A.n;
    const int tiles_x = (int)((n + 1 + T::TC - 1) / T::TC);
    const int tiles_y = (int)((A.rb - A.ra + T::TR - 1) / T::TR);
    const long grid = (long)tiles_x * tiles_y;
    if ((MODE & 8) && grid > kNormBlocks) return -1;
    if (A.c.fm)
        MGX_LAUNCH((k_smooth_tile<K, MODE, TRV, true>), dim3((unsigned)grid), dim3(T::THREADS), s,
                   A.uin, A.uout, A.rhs, A.v1, A.v2, A.uc, A.pitchc, A.rhsc, A.partials, (int)n,
                   A.pitch, tiles_x, A.c, A.ra, A.rb, A.lo, A.hi, g_tile_xcd ? 1 : 0, A.cf);
    else
        MGX_LAUNCH((k_smooth_tile<K, MODE, TRV, false>), dim3((unsigned)grid), dim3(T::THREADS), s,
                   A.uin, A.uout, A.rhs, A.v1, A.v2, A.uc, A.pitchc, A.rhsc, A.partials, (int)n,
                   A.pitch, tiles_x, A.c, A.ra, A.rb, A.lo, A.hi, g_tile_xcd ? 1 : 0, A.cf);
    return (int)grid;
}

// 16 x 64 output tiles (halo overhead 2.5x the tile); with K = 3 on levels
// n >= tile32_min_n, 32 x 64 (1.9x, more work per workgroup)
template <int K, int MODE>
static int smooth_tile_inst(const SmoothArgs &A, hipStream_t s) {
    if constexpr (K == 3)
        if (A.n >= g_tile32_min_n) return smooth_tile_rows<K, MODE, 32>(A, s);
    return smooth_tile_rows<K, MODE, 16>(A, s);
}

// a row block runs as LDS tiles when its march would give the resident waves
// fewer than this many rows each (tuning key "march_tile_rows"; 16: level 2
// on 4 row blocks marches, 0.50 -> 0.46 ms for the 4 parts; level 1 on 8 row
// blocks as tiles (64, 96) costs +25-45 %)
long g_march_tile_rows = 16;
void set_march_tile_rows(long v) { g_march_tile_rows = v; }
long get_march_tile_rows() { return g_march_tile_rows; }

// whether the pass runs as LDS tiles (else the wave-private row march)
template <int K, int MODE>
static bool smooth_as_tiles(const SmoothArgs &A) {
    // the row march needs >= ~32 rows per wave to amortise its priming rows;
    // a row block too small to give every resident wave that much (a
    // partitioned level on many GPUs) runs as LDS tiles instead
    bool tile = A.n <= g_tile_max_n && !(MODE & 16);   // RHSN: march only
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
    return tile;
}

template <int K, int MODE>
static int smooth_block(const SmoothArgs &A, hipStream_t s) {
    const bool tile = smooth_as_tiles<K, MODE>(A);
    // a fused coarse solve needs the tile pass (the march reads uc from HBM)
    const bool fused = A.cf.on && (MODE & kModeProlong) && A.cf.n <= kCoarseLdsMaxN;
    if (A.cf.on && !fused) return -4;
    if (tile) {
        const int g = smooth_tile_inst<K, MODE>(A, s);
        if (g > 0) return g;
    }
    if (fused) return -4;
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

bool smooth_generates_velocity(const SmoothArgs &A0, int sweeps, int mode) {
    if (!A0.vg.a || sweeps != 3) return false;
    SmoothArgs A = A0;   // (the whole level: as launch_smooth)
    if (A.rb < 0) {
        A.ra = 0;
        A.rb = (int)A.n + 1;
    }
    if (mode == (kModeZero | kModeRestrict)) return !smooth_as_tiles<3, kModeZero | kModeRestrict>(A);
    if (mode == kModeProlong) return !smooth_as_tiles<3, kModeProlong>(A);
    if (mode == kModeRestrict) return !smooth_as_tiles<3, kModeRestrict>(A);
    return false;
}

// A W-cycle's two adjacent smoothing passes of one tile level (the post-
// smoothing of visit sh and the pre-smoothing of visit sh+1, multigrid.cpp:
// 52, 69-88: nothing runs between them) as ONE LDS-tile pass: prolongation +
// add, 2*nsmooth sweeps, residual restricted -- the same operations in the same
// order as the two passes, so bitwise their result; one launch and one
// stage chain instead of two.  Tiles only (the small, latency-bound levels,
// where the 2x wider halo costs nothing that matters): -1 when the level
// would march, or for nsmooth outside 1..3.
int launch_smooth_wpair(const SmoothArgs &A0, int nsmooth, hipStream_t s) {
    SmoothArgs A = A0;
    if (A.rb < 0) {
        A.ra = 0;
        A.rb = (int)A.n + 1;
        A.lo = 0;
        A.hi = (int)A.n;
    }
    if (A.ra & 1) return -1;
    if (A.cf.on && A.cf.n > kCoarseLdsMaxN) return -4;
    constexpr int M = kModeProlong | kModeRestrict;
    switch (nsmooth) {
        case 1:
            if (!smooth_as_tiles<1, M>(A)) return -1;
            return smooth_tile_rows<2, M, 16>(A, s);
        case 2:
            if (!smooth_as_tiles<2, M>(A)) return -1;
            return smooth_tile_rows<4, M, 16>(A, s);
        case 3:
            if (!smooth_as_tiles<3, M>(A)) return -1;
            return smooth_tile_rows<6, M, 16>(A, s);
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
        launch_norm_final(A.partials, blocks, A.norm_out, A.norm_accumulate ? 2 : A.norm_sqrt ? 1 : 0, s);
    return blocks;
}

}  // namespace mgx
