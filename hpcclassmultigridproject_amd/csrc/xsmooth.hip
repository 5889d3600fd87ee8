// xsmooth.hip -- the finest level's cross-cycle pass: post-smoothing of
// V-cycle k fused with the pre-smoothing of cycle k+1 (k_xsmooth, a row march
// of wave pairs), its LDS-tile form for short row blocks (k_xtile), and
// launch_xsmooth.
#include "stencil.h"

namespace mgx {
namespace {

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
// FM = true (fp_mode fma, stencil.h): each row's rhs enters the ring as f' =
// f/d at its first use (A: the row's first stage, before the hand-off, so B
// receives it scaled), the per-row coefficients are the m = -c/d of the
// contracted update (one fma each), every update is four fmas and every
// residual d*(update - u).  B's time-step rhs (RS) keeps the reference
// expressions (gs.cpp:44, stored unscaled) and is scaled after.
template <int WPB, int K, bool G, bool RS = false, bool SV = false, bool FM = false>
__global__ __launch_bounds__(128 * WPB) void k_xsmooth(
    const double *__restrict__ uin, double *__restrict__ upost, double *__restrict__ upre,
    const double *__restrict__ rhs, const double *__restrict__ v1, const double *__restrict__ v2,
    const double *__restrict__ uc, long pitchc, double *__restrict__ rhsc,
    double *__restrict__ partials, int n, long pitch, MarchRegions reg, long units_per_wg, Coef c,
    int lo, int hi, int store_post, double *__restrict__ rhs_next,
    double *__restrict__ partials2, const double *__restrict__ sa1,
    const double *__restrict__ sb1, const double *__restrict__ sa2,
    const double *__restrict__ sb2) {
    using X = XCfg<K>;
    constexpr int S = X::S, H = X::H, NR = X::NR, W = X::W, D = X::D, NU = X::NU,
                  NRD = X::NRD, EA = X::EA, EB = X::EB;
    // A's prefetch distances in steps: rhs/v rows XRV ahead of their first
    // stage, u rows (+ coarse parents) XU ahead of entering the ring.  The
    // pass is bound by loads in flight, not by VALU: rhs/v 2 -> 3 -> 4 steps
    // took level 0 -4 % and -3 % at the same VGPR count (B's path sets it);
    // u 3-4 steps or rhs/v 5 measured no better (N=16384, tools/ab_libs.sh).
    // (the fma interior kernel on the velocity factors: 5 steps, -0.8 % on
    // level 0 in three alternated rounds, 2 VGPRs spilled; XU 3 no change)
    constexpr int XRV = (FM && SV && !G && !RS) ? MGX_XRV + 1 : MGX_XRV;
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
        const bool keep = act && c0 >= k0 && c0 < k1;
        // (rows [a, b) as one unsigned compare: b >= a)
        auto own = [&](const int r) { return (unsigned)(r - a) < (unsigned)(b - a) && keep; };
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
        double2 ur[NR];   // u rows (ring by row)
        // u rows + coarse parents in flight, a ring by row like rd
        UPre up[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            up[i] = UPre{make_double2(0.0, 0.0), 0.0, 0.0, 0.0, 0.0};
            ur[i] = make_double2(0.0, 0.0);
            rd[i].r = rd[i].x = rd[i].y = make_double2(0.0, 0.0);
        }
        // A: u row R + its coarse parents (odd = R's parity, compile-time:
        // an even row needs only the coarse row below it)
        auto load_u = [&](int R, UPre &u, const bool odd) {
            const int Rc = min(max(R, lo), hi);
            u.X = ld2u(uin + rowoff(Rc, ip), bcl);
            const double *p0 = uc + rowoff(Rc >> 1, ipc);
            u.q00 = ld1u(p0, bjl);
            u.q01 = ld1u(p0, bjl1);
            if (odd) {   // (a row clamped to an even one: its own parent, never past hi)
                const double *p1 = p0 + ((Rc & 1) ? ipc : 0);
                u.q10 = ld1u(p1, bjl);
                u.q11 = ld1u(p1, bjl1);
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
        // A, the row in slot q at its first stage: t from the factors (SV),
        // and f' = f/d (FM)
        auto first_use = [&](const int q) {
            if (SV) {
                rd[q].x = make_double2(ar1[q] * bh1.x, ar1[q] * bh1.y);
                rd[q].y = make_double2(ar2[q] * bh2.x, ar2[q] * bh2.y);
            }
            if (FM) rd[q].r = make_double2(rd[q].r.x * c.rdgs, rd[q].r.y * c.rdgs);
        };
        // one red-black stage h of the march step at row phase p on row r,
        // the coefficients from t (A's stages in the guarded kernel)
        auto stage = [&](const int p, const int h, const int r) {
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
                const double uW = dpp_shr1(ur[iR].y);
                if (!GS || (inr && in0))
                    ur[iR].x = FM ? fm_upd_t(d.r.x, d.x.x, d.y.x, ur[iN].x, uW, ur[iS].x,
                                             ur[iR].y, c)
                                  : gs_point_t<!GS>(d.r.x, d.x.x, d.y.x, ur[iN].x, uW, ur[iS].x,
                                                    ur[iR].y, cg);
            } else {
                const double uE = dpp_shl1(ur[iR].x);
                if (!GS || (inr && in1))
                    ur[iR].y = FM ? fm_upd_t(d.r.y, d.x.y, d.y.y, ur[iN].y, ur[iR].x, ur[iS].y,
                                             uE, c)
                                  : gs_point_t<!GS>(d.r.y, d.x.y, d.y.y, ur[iN].y, ur[iR].x,
                                                    ur[iS].y, uE, cg);
            }
        };
        // residual of the row in slot iR at column c0 / c0+1 from its t
        // (gs.cpp:75 term order; FM: d*(update - u))
        auto res_tx = [&](const int iR, const int iN, const int iS, const double uW) {
            const RowData &d = rd[iR];
            return FM ? fm_res_t(d.r.x, d.x.x, d.y.x, ur[iR].x, ur[iN].x, uW, ur[iS].x, ur[iR].y,
                                 c)
                      : res_point_t(d.r.x, d.x.x, d.y.x, ur[iR].x, ur[iN].x, uW, ur[iS].x,
                                    ur[iR].y, c);
        };
        auto res_ty = [&](const int iR, const int iN, const int iS, const double uE) {
            const RowData &d = rd[iR];
            return FM ? fm_res_t(d.r.y, d.x.y, d.y.y, ur[iR].y, ur[iN].y, ur[iR].x, ur[iS].y, uE,
                                 c)
                      : res_point_t(d.r.y, d.x.y, d.y.y, ur[iR].y, ur[iN].y, ur[iR].x, ur[iS].y,
                                    uE, c);
        };

        // A's first step (aligned to NR so ring indices and parities are
        // static); B runs D steps behind; the last iteration is B's last step
        // (rounded up to whole pairs: an extra step stores nothing)
        int s0 = a - EB - EA - (RS ? 1 : 0);
        s0 = s0 >= 0 ? (s0 / NR) * NR : -(((-s0) + NR - 1) / NR) * NR;
        s0 = __builtin_amdgcn_readfirstlane(s0);
        const int iters = ((b + EB - 3) + D - s0 + 1 + 1) & ~1;
        const bool post = store_post != 0;

        // B turns each rhs/v row's t1, t2 into the four coefficients of its
        // two points once (gs.cpp:126-129, the expressions of gs_point_t),
        // just before the row's first stage, instead of in each of the
        // point's three stages and its restriction residual: -12 % VALU per
        // pass, -3 % time (the same in A as well: -23 % VALU, no further
        // time, 254 instead of 224 VGPRs -- the pass is not issue bound)
        // (FM: the m = -c/d of the contracted update)
        CoefRow cf[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const double2 z = make_double2(0.0, 0.0);
            cf[i] = CoefRow{z, z, z, z};
        }
        auto to_coef = [&](const RowData &d, CoefRow &k) {
            if (FM) {
                k.cn = make_double2(fm_mp(d.x.x, c), fm_mp(d.x.y, c));
                k.cw = make_double2(fm_mp(d.y.x, c), fm_mp(d.y.y, c));
                k.cs = make_double2(fm_ms(k.cn.x, c), fm_ms(k.cn.y, c));
                k.ce = make_double2(fm_ms(k.cw.x, c), fm_ms(k.cw.y, c));
                return;
            }
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
                const double uW = dpp_shr1(ur[iR].y);
                if (!GS || (inr && in0))
                    ur[iR].x = FM ? fm_upd(f.x, k.cn.x, ur[iN].x, k.cw.x, uW, k.cs.x, ur[iS].x,
                                           k.ce.x, ur[iR].y)
                                  : div_diag<!GS>(f.x - k.cn.x * ur[iN].x - k.cw.x * uW -
                                                      k.cs.x * ur[iS].x - k.ce.x * ur[iR].y,
                                                  c);
            } else {
                const double uE = dpp_shl1(ur[iR].x);
                if (!GS || (inr && in1))
                    ur[iR].y = FM ? fm_upd(f.y, k.cn.y, ur[iN].y, k.cw.y, ur[iR].x, k.cs.y,
                                           ur[iS].y, k.ce.y, uE)
                                  : div_diag<!GS>(f.y - k.cn.y * ur[iN].y - k.cw.y * ur[iR].x -
                                                      k.cs.y * ur[iS].y - k.ce.y * uE,
                                                  c);
            }
        };
        // residual (gs.cpp:75 term order) at column c0 of the row in slot iR,
        // from its coefficients
        auto res_x = [&](const int iR, const int iN, const int iS, const double uW) {
            const CoefRow &k = cf[iR];
            if (FM)
                return fm_res(rd[iR].r.x, ur[iR].x, k.cn.x, ur[iN].x, k.cw.x, uW, k.cs.x,
                              ur[iS].x, k.ce.x, ur[iR].y, c);
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
                    first_use((p + 1) % NR);   // row s+1: first used by stage 0 below
                    if (XACOEF) {
                        // the row's four coefficients once (as B does), not in
                        // each of its point's stages
                        to_coef(rd[(p + 1) % NR], cf[(p + 1) % NR]);
#pragma unroll
                        for (int h = 0; h < S; ++h) stage_c(p, h, s + 1 - h);
                    } else {
#pragma unroll
                        for (int h = 0; h < S; ++h) stage(p, h, s + 1 - h);
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
                        st2_ifu(upost + rowoff(ro, ip), c0, post && own(ro), uf);
                    }
                    // residual norm of u_post (multigrid.cpp:112-113), column c0 of
                    // row s+1-S (its neighbours are final now; B takes column c0+1:
                    // half each balances the pair's VALU work)
                    {
                        const int r = s + 1 - S;
                        const int iR = (p + 1 - S + 2 * NR) % NR;
                        const int iN = (p - S + 2 * NR) % NR;
                        const int iS = (p + 2 - S + 2 * NR) % NR;
                        const double uW = dpp_shr1(ur[iR].y);
                        // (with the row's coefficients: the same expressions, bitwise)
                        auto res0 = [&]() {
                            if (XACOEF) return res_x(iR, iN, iS, uW);
                            return res_tx(iR, iN, iS, uW);
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
                    if (p & 1) {   // end of a pair (compile-time)
                        __syncthreads();
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
                        const double uE = dpp_shl1(ur[iR].x);
                        if (GN) {
                            if (own(r) && r >= 1 && r <= n - 1 && in1) {
                                const double res = res_ty(iR, iN, iS, uE);
                                acc += res * res;
                            }
                        } else {   // acc + 0.0 == acc (acc >= +0): a select, no branch
                            const double r1 = res_ty(iR, iN, iS, uE);
                            acc += own(r) ? r1 * r1 : 0.0;
                        }
                    }
                    if (RS) {
                        // the next step's rhs of row s+2 from u_post rows s+1..s+3
                        // (gs.cpp:44), stored on the owned interior points, and the
                        // residual of u_post against it (multigrid.cpp:104); it
                        // replaces this step's rhs in the ring for B's stages and
                        // restriction (FM: scaled to f/d after)
                        const int r = s + 2;
                        const int iR = (q + 2) % NR, iN = (q + 1) % NR, iS = (q + 3) % NR;
                        RowData &d = rd[iR];
                        const double uW = dpp_shr1(ur[iR].y), uE = dpp_shl1(ur[iR].x);
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
                        if (FM) d.r = make_double2(f0 * c.rdgs, f1 * c.rdgs);
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
                        const double uW = dpp_shr1(ur[iR].y);
                        const bool on = own(r) &&
                                        (!GN || (r >= 1 && r <= n - 2 && in0 && c0 <= n - 2));
                        const double res = res_x(iR, iN, iS, uW);
                        st1_ifu(rhsc + rowoff(r >> 1, ipc), c0 >> 1, on, res);
                    }
                    if (p & 1) {
                        __syncthreads();
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
        if (__builtin_amdgcn_readfirstlane(strip) >= 0)
            march(strip * W - 2 * H, strip * W, strip * W + W, a, b);
    }
    const double tot = wave_sum(acc);   // one partial per wave (A: columns c0, B: c0+1)
    if (l == 0) partials[(long)blockIdx.x * 2 * WPB + wv] = tot;
    if (RS) {
        const double tot2 = wave_sum(acc2);   // B only (A's are +0)
        if (l == 0) partials2[(long)blockIdx.x * 2 * WPB + wv] = tot2;
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

// FM: fp_mode fma (stencil.h): the pair keeps f' = f/d and the m = -c/d of
// the contracted update instead.
template <int K, int TRV, bool FM>
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
            const double hh = c.h * 0.5;   // FM: from t = v*h/2 (stencil.h)
            auto fmc = [&](double f, double t1, double t2) {
                const double mn = fm_mp(t1, c), mw = fm_mp(t2, c);
                return PtCoef{f * c.rdgs, mn, mw, fm_ms(mn, c), fm_ms(mw, c)};
            };
            const PtCoef X = FM ? fmc(rr.x, xx.x * hh, yy.x * hh)
                                : PtCoef{rr.x, coef_a(xx.x, c), coef_a(yy.x, c), coef_b(xx.x, c),
                                         coef_b(yy.x, c)};
            const PtCoef Y = FM ? fmc(rr.y, xx.y * hh, yy.y * hh)
                                : PtCoef{rr.y, coef_a(xx.y, c), coef_a(yy.y, c), coef_b(xx.y, c),
                                         coef_b(yy.y, c)};
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
                ow[q] = FM ? fm_upd(P.f, P.cn, uN, P.cw, uW, P.cs, uS, P.ce, uE)
                           : div_diag(P.f - P.cn * uN - P.cw * uW - P.cs * uS - P.ce * uE, c);
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
        if (FM)
            return fm_res(P.f, pu[q], P.cn, ot[q - HW], P.cw, ot[q - 1 + cs], P.cs, ot[q + HW],
                          P.ce, ot[q + cs], c);
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

}  // namespace

long g_xfast = 1;   // unguarded interior march kernels (tuning key "xfast")
void set_xfast(long v) { g_xfast = v; }
long get_xfast() { return g_xfast; }

template <int WPB, int K, bool G, bool RS, bool SV, bool FM>
static int xsmooth_slots() {
    static int slots = 0;   // resident workgroups of this instantiation
    if (!slots) {
        int dev = 0, cus = 0, per = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per,
                                                           k_xsmooth<WPB, K, G, RS, SV, FM>,
                                                           128 * WPB, 0);
        slots = std::max(1, cus) * std::max(1, per);
    }
    return slots;
}

// One launch over `reg`; min_rows: the fewest rows per workgroup (each
// workgroup's march pays a warm-up of ~EA + EB + D rows).  Returns the norm
// partials written (grid * 2 * WPB: one per wave) at `partials`.
template <int WPB, int K, bool G, bool RS, bool SV, bool FM>
static int xsmooth_launch_sv(const XArgs &A, const MarchRegions &reg, double *partials, int lo,
                             int hi, long min_rows, long max_wgs, hipStream_t s) {
    const long total = reg.pre[reg.count];
    if (total <= 0) return 0;
    long upw;
    MarchRegions r;
    using X = XCfg<K>;
    const unsigned grid = plan_march(reg, WPB, xsmooth_slots<WPB, K, G, RS, SV, FM>(), min_rows,
                                     max_wgs, X::EA + X::EB + X::D + X::NR / 2, upw, r);
    // RS: the second partials (the next step's initial norm) at the same
    // offsets, kNormBlocks further on
    MGX_LAUNCH((k_xsmooth<WPB, K, G, RS, SV, FM>), dim3(grid), dim3(128 * WPB), s, A.uin,
               A.upost, A.upre, A.rhs, A.v1, A.v2, A.uc, A.pitchc, A.rhsc, partials, (int)A.n,
               A.pitch, r, upw, A.c, lo, hi, A.store_post ? 1 : 0, A.rhs_next,
               RS ? partials + kNormBlocks : (double *)nullptr, A.sa1, A.sb1, A.sa2, A.sb2);
    return (int)grid * 2 * WPB;
}
// SV when the level's velocity factors are given (XArgs::sa1); FM = the
// level's fp_mode (Coef::fm)
template <int WPB, int K, bool G, bool RS = false>
static int xsmooth_launch(const XArgs &A, const MarchRegions &reg, double *partials, int lo, int hi,
                          long min_rows, long max_wgs, hipStream_t s) {
    const bool sv = A.sa1 && A.sb1 && A.sa2 && A.sb2;
    if (A.c.fm) {
        if (sv)
            return xsmooth_launch_sv<WPB, K, G, RS, true, true>(A, reg, partials, lo, hi,
                                                               min_rows, max_wgs, s);
        return xsmooth_launch_sv<WPB, K, G, RS, false, true>(A, reg, partials, lo, hi, min_rows,
                                                            max_wgs, s);
    }
    if (sv)
        return xsmooth_launch_sv<WPB, K, G, RS, true, false>(A, reg, partials, lo, hi, min_rows,
                                                            max_wgs, s);
    return xsmooth_launch_sv<WPB, K, G, RS, false, false>(A, reg, partials, lo, hi, min_rows,
                                                         max_wgs, s);
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

template <int K, int TRV>
static void xtile_launch(const XArgs &A, const TileRegions &t, int tiles, double *partials, int lo,
                         int hi, hipStream_t s) {
    if (A.c.fm)
        MGX_LAUNCH((k_xtile<K, TRV, true>), dim3((unsigned)tiles), dim3(256), s, A.uin, A.upre,
                   A.upost, A.rhs, A.v1, A.v2, A.uc, A.pitchc, A.rhsc, partials, (int)A.n, A.pitch,
                   t, A.c, lo, hi, A.store_post ? 1 : 0);
    else
        MGX_LAUNCH((k_xtile<K, TRV, false>), dim3((unsigned)tiles), dim3(256), s, A.uin, A.upre,
                   A.upost, A.rhs, A.v1, A.v2, A.uc, A.pitchc, A.rhsc, partials, (int)A.n, A.pitch,
                   t, A.c, lo, hi, A.store_post ? 1 : 0);
}

template <int WPB, int K>
static int xsmooth_tiled(const XArgs &A, int ra, int rb, int lo, int hi, hipStream_t s) {
    using X = XCfg<K>;
    const long n = A.n;
    int si0, si1, ma, mb, top, bot;
    xmargins<K>(A, ra, rb, top, bot);
    march_split(n, X::W, X::H, ra, rb, top, bot, si0, si1, ma, mb);
    TileRegions t{};
    const bool inner_march = si1 > si0 && mb - ma >= kXTileAllRows;
    if (inner_march) {
        const int ca = si0 * X::W;
        const int cb = (int)std::min<long>(n + 1, (long)si1 * X::W);
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
        MarchRegions inner{};
        add_region<WPB>(inner, si0, si1, ma, mb);
        pm = xsmooth_launch<WPB, K, false>(A, inner, A.partials, lo, hi, A.min_rows,
                                           kNormBlocks / (2 * WPB) / 2, s);
    }
    if (A.phase == 1) return pm;
    if (tiles > 0) xtile_launch<K, kXTileRows>(A, t, tiles, A.partials + pm, lo, hi, s);
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
    march_regions<WPB>(n, X::W, X::H, ra, rb, top, bot, split, inner, unused);
    march_regions<1>(n, X::W, X::H, ra, rb, top, bot, split, unused, edge);
    int pm = A.partials_done;
    if (A.phase != 2)
        pm = xsmooth_launch<WPB, K, false>(A, inner, A.partials, lo, hi, A.min_rows,
                                           kNormBlocks / (2 * WPB) / 2, s);
    if (A.phase == 1) return pm;
    const int pe = xsmooth_launch<1, K, true>(A, edge, A.partials + pm, lo, hi,
                                              std::min(MGX_XEDGE_ROWS, A.min_rows),
                                              kNormBlocks / 2 / 2, s);
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
        launch_norm_final(A.partials, blocks, A.norm_out, A.norm_accumulate ? 2 : A.norm_sqrt ? 1 : 0, s);
    if (blocks > 0 && A.rhs_next)   // the next step's initial norm
        launch_norm_final(A.partials + kNormBlocks, blocks, A.norm2_out, 1, s);
    return blocks;
}

bool xstep_supported(long n) {
    return g_xfast != 0 && n + 1 > g_xtile_max_rows;
}

}  // namespace mgx
