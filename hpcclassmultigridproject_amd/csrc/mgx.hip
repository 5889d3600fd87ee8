// mgx.hip -- context, V-cycle orchestration and the C ABI of include/mgx.h.
//
// Host control flow mirrors the reference solver (multigrid.cpp:17-186) call
// for call; every stencil op is a CDNA4 kernel from kernels.hip on the
// context's stream.  The level towers live in HBM in the "tower layout"
// (row pitch round_up(n+1,16) doubles); u has two buffers per level because
// the one-pass smoother is out of place (ping-pong).  Row-partitioned
// multi-GPU contexts (ctx->dist) are implemented in dist.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "ctx.h"
#include "sepvel.h"

namespace mgxi {

thread_local std::string g_err;

// tuning key "sep_velocity": 1 (default) = at upload, a velocity field that is
// an exact rank-1 outer product (the reference's rotating flow) is also kept
// as its factors and the finest-level cross pass reads those instead of the
// 2-D v1 / v2 (sepvel.h; bitwise the same results); 0 = always the 2-D arrays
long g_sep_velocity = 1;

bool factor_velocity(const double *v1, const double *v2, long n, long r0, long rows, double smin,
                     std::vector<double> &a1, std::vector<double> &b1, std::vector<double> &a2,
                     std::vector<double> &b2, long *js1, long *js2) {
    (void)r0;
    if (!g_sep_velocity || !v1 || !v2 || rows < 1) return false;
    const long w = n + 1;
    a1.assign(rows, 0.0);
    a2.assign(rows, 0.0);
    b1.assign(w, 0.0);
    b2.assign(w, 0.0);
    return mgxsep::factor_rank1(v1, rows, w, w, smin, a1.data(), b1.data(), 0, js1) &&
           mgxsep::factor_rank1(v2, rows, w, w, smin, a2.data(), b2.data(), 0, js2);
}

void free_level_factors(Level &L) {
    for (double **p : {&L.sa1, &L.sb1, &L.sa2, &L.sb2}) {
        (void)hipFree(*p);
        *p = nullptr;
    }
}

// Device copies: row factors at rows [row0, row0 + a.size()) of an (n+1)-row
// array (the rest zero), column factors zero padded to the pitch.
int set_level_factors(Level &L, long row0, const std::vector<double> &a1,
                      const std::vector<double> &b1, const std::vector<double> &a2,
                      const std::vector<double> &b2, hipStream_t s) {
    free_level_factors(L);
    const size_t ra = sizeof(double) * (size_t)(L.n + 1), rb = sizeof(double) * (size_t)L.pitch;
    HIPCHK(hipMalloc(&L.sa1, ra));
    HIPCHK(hipMalloc(&L.sa2, ra));
    HIPCHK(hipMalloc(&L.sb1, rb));
    HIPCHK(hipMalloc(&L.sb2, rb));
    for (double *p : {L.sa1, L.sa2}) HIPCHK(hipMemsetAsync(p, 0, ra, s));
    for (double *p : {L.sb1, L.sb2}) HIPCHK(hipMemsetAsync(p, 0, rb, s));
    HIPCHK(hipMemcpyAsync(L.sa1 + row0, a1.data(), sizeof(double) * a1.size(),
                          hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(L.sa2 + row0, a2.data(), sizeof(double) * a2.size(),
                          hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(L.sb1, b1.data(), sizeof(double) * b1.size(), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(L.sb2, b2.data(), sizeof(double) * b2.size(), hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));   // the host vectors may go out of scope
    return MGX_OK;
}

// Cross-cycle fusion of the finest level (k_xsmooth) on levels this large
// (the row-march regime); tuning key "cross_cycle" turns it off.
long g_cross_cycle = 1;
bool cross_cycle_on() { return g_cross_cycle != 0; }

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MGX_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return MGX_OK;
}

hipEvent_t take_event(mgx_ctx *c) {
    if (!c->pool.empty()) {
        hipEvent_t e = c->pool.back();
        c->pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

int prof_flush(mgx_ctx *c) {
    if (c->pending.empty()) return MGX_OK;
    HIPCHK(hipStreamSynchronize(c->stream));
    for (auto &r : c->pending) {
        float ms = 0.f;
        // (a partitioned context times its side-stream exchanges too)
        HIPCHK(hipEventSynchronize(r.e1));
        HIPCHK(hipEventElapsedTime(&ms, r.e0, r.e1));
        int lvl = r.level < 0 ? 0 : (r.level > 63 ? 63 : r.level);
        c->sum_ms[r.kind][lvl] += ms;
        c->sum_bytes[r.kind][lvl] += r.bytes;
        c->sum_cbytes[r.kind][lvl] += r.cbytes;
        c->count[r.kind][lvl] += 1;
        c->pool.push_back(r.e0);
        c->pool.push_back(r.e1);
    }
    c->pending.clear();
    return MGX_OK;
}

// ---------------------------------------------------------------- level ops
int materialize(mgx_ctx *c, int l) {
    Level &L = c->lv[l];
    if (!L.zero) return MGX_OK;
    HIPCHK(hipMemsetAsync(L.U(), 0, sizeof(double) * L.pitch * (L.n + 1), c->stream));
    L.zero = false;
    return MGX_OK;
}

// `sweeps` RB-GS sweeps (gauss_seidel, gs.cpp:109) on level l.
//   prolong:  first apply u[l] += P(u[l+1]) (multigrid.cpp:81-83);
//   restrict: afterwards restrict the residual into rhs[l+1] (multigrid.cpp:73-75);
//   norm:     afterwards compute the residual norm into c->dscal[0].
// With the temporally blocked smoother all three are fused into the first /
// last smoothing pass; *fused_norm tells the caller whether the norm was done.
int op_prolong_add(mgx_ctx *c, int l);
int op_restrict(mgx_ctx *c, int l);
// tuning key "vgen": 1 (default) = levels 1-2 of the reference tower and
// every coarse level of the correct tower, when their velocity passed the
// upload check (find_vgen), generate v1 / v2 in the V-cycle's 3-sweep passes
// from the finest factors instead of reading them (stencil.h vg_col; bitwise
// the same); 0 = reads them
long g_vgen = 1;
static mgx::VGen level_vgen(const mgx_ctx *c, int l) {
    mgx::VGen g;
    g.a = c->vga;
    g.b1 = c->lv[0].sb1;
    g.b2 = c->lv[0].sb2;
    g.l = l;
    g.strided = c->opt.tower_mode == MGX_TOWER_CORRECT ? 1 : 0;
    return g;
}
// tuning key "coarse_fuse": 1 (default) = the coarsest solve (n <= 64, u in
// LDS) runs inside the prolongation tile pass of the level above: every
// workgroup of that pass solves the coarsest level in its LDS and prolongs
// from the copy (mgx::CoarseFuse), one launch less per visit -- bitwise the
// same; 0 = its own launch (op_coarse)
long g_coarse_fuse = 1;
int op_coarse(mgx_ctx *c, int l, int reps);
// (only from a zero start, the V- and W-cycle's case after the restriction:
// then no workgroup reads the coarse u that workgroup 0 stores at its end;
// and only with nsmooth >= 1, so that the post-smoothing above is a tile pass
// that can take it -- nsmooth 0 prolongs with op_prolong_add)
static bool coarse_fusable(const mgx_ctx *c, int l) {
    return g_coarse_fuse && !c->dist && c->opt.smoother == 0 && c->opt.nsmooth >= 1 &&
           l == c->L - 1 && l >= 2 && c->lv[l].zero &&
           c->lv[l].n <= mgx::kCoarseLdsMaxN && mgx::get_coarse_lds() &&
           c->lv[l - 1].n <= mgx::get_tile_max_n();
}
// run a pending fused coarsest solve on its own (its consumer cannot take it)
static int flush_coarse(mgx_ctx *c) {
    if (c->cf_level < 0) return MGX_OK;
    const int l = c->cf_level;
    c->cf_level = -1;
    return op_coarse(c, l, c->cf_reps);
}
// A pass that restricts into the rhs its fused coarsest solve reads would race
// (every workgroup loads cf.rhs at its start while others already store the
// restriction): refuse it.  mode: the pass's kMode bits.
static int check_coarse_rhs(const mgx::SmoothArgs &A, int mode) {
    if (A.cf.on && (mode & mgx::kModeRestrict) && A.rhsc == A.cf.rhs)
        return fail(MGX_E_INTERNAL, "fused coarsest solve reads the rhs its pass restricts into");
    return MGX_OK;
}
// the pending coarsest solve of level l+1 into a prolongation pass of level l
static bool take_coarse(mgx_ctx *c, int l, mgx::SmoothArgs &A) {
    if (c->cf_level != l + 1) return false;
    Level &Cl = c->lv[l + 1];
    A.cf.u = Cl.U();
    A.cf.rhs = Cl.rhs;
    A.cf.v1 = Cl.v1;
    A.cf.v2 = Cl.v2;
    A.cf.n = Cl.n;
    A.cf.pitch = Cl.pitch;
    A.cf.c = Cl.coef;
    A.cf.tol = c->opt.coarse_tol;
    A.cf.maxit = c->opt.coarse_maxit;
    A.cf.zero_first = Cl.zero ? 1 : 0;
    A.cf.reps = c->cf_reps;
    A.cf.stats = c->dscal + 2;
    A.cf.on = 1;
    return true;
}
// after a launch that took it: the coarse level holds its solution
static void took_coarse(mgx_ctx *c, int l) {
    c->cf_level = -1;
    c->lv[l + 1].zero = false;
}

int op_smooth(mgx_ctx *c, int l, int sweeps, bool prolong, bool restrict_, bool norm,
              bool *fused_norm) {
    Level &L = c->lv[l];
    if (fused_norm) *fused_norm = false;
    if (c->opt.smoother == 0 && sweeps > 0) {
        const int fuse = std::max(1, std::min(c->opt.fuse, mgx::kSmoothMaxSweeps));
        int done = 0;
        while (done < sweeps) {
            const int k = std::min(sweeps - done, fuse);
            const bool first = done == 0, last = done + k == sweeps;
            const bool pr = prolong && first && !L.zero;
            const bool rs = restrict_ && last;
            const bool nm = norm && last && !rs;
            // a pending coarsest solve of level l+1 runs inside this pass
            // (its u is then not read from HBM: no zero fill either)
            const bool cfuse = pr && c->cf_level == l + 1;
            if (pr && !cfuse) CHK(materialize(c, l + 1));
            int mode = 0;
            if (L.zero) mode |= mgx::kModeZero;
            if (pr) mode |= mgx::kModeProlong;
            if (rs) mode |= mgx::kModeRestrict;
            if (nm) mode |= mgx::kModeNorm;
            mgx::SmoothArgs A{};
            A.uin = L.u[L.cur];
            A.uout = L.u[L.nxt()];
            A.rhs = L.rhs;
            A.v1 = L.v1;
            A.v2 = L.v2;
            A.zrow = c->zrow;
            A.vz = L.vz;
            if (L.vgen && g_vgen) A.vg = level_vgen(c, l);
            A.n = L.n;
            A.pitch = L.pitch;
            A.c = L.coef;
            if (pr || rs) {
                Level &Cl = c->lv[l + 1];
                A.uc = Cl.U();
                A.rhsc = Cl.rhs;
                A.pitchc = Cl.pitch;
            }
            A.partials = c->partials;
            A.norm_out = c->dscal;
            if (cfuse) take_coarse(c, l, A);
            double bytes = 40.0 * k * L.M();
            int kind = MGX_K_GS;
            if (pr) {
                bytes += 32.0 * L.M() + 8.0 * c->lv[l + 1].M();
                kind = MGX_K_PSMOOTH;
            }
            if (rs) bytes += 40.0 * L.M() + 24.0 * c->lv[l + 1].M();
            if (nm) bytes += 48.0 * L.M();
            // compulsory: u (unless zero), rhs, v1, v2 read, u written, the
            // coarse u read (prolong) / coarse rhs written (restrict)
            // (v1 / v2 rows >= vz come from the zero row, not HBM)
            // (generated velocity: the 3-sweep pre / post marches, launch_smooth)
            const bool vgu = mgx::smooth_generates_velocity(A, k, mode);
            const double cbytes = 8.0 * (((mode & mgx::kModeZero) ? 2.0 : 3.0) * L.M() +
                                         (vgu ? 0.0 : 2.0 * L.Mv()) +
                                         ((pr ? 1 : 0) + (rs ? 1 : 0)) * c->lv[l + 1].M());
            int blocks = 0;
            CHK(check_coarse_rhs(A, mode));
            const size_t before = c->pending.size();
            CHK(launch(c, kind, l, bytes, cbytes,
                       [&] { blocks = mgx::launch_smooth(A, k, mode, c->stream); }));
            if (blocks < 0) unlaunch(c, before);
            if (blocks == -4 && cfuse) {
                // the pass would march: the coarsest solve on its own, then the pass
                // (nothing was launched)
                A.cf = mgx::CoarseFuse{};
                CHK(flush_coarse(c));
                A.uc = c->lv[l + 1].U();
                CHK(launch(c, kind, l, bytes, cbytes,
                           [&] { blocks = mgx::launch_smooth(A, k, mode, c->stream); }));
            } else if (cfuse) {
                took_coarse(c, l);
            }
            if (blocks < 0) return fail(MGX_E_ARG, "launch_smooth: unsupported sweeps/mode");
            L.cur = L.nxt();
            L.zero = false;
            if (rs) c->lv[l + 1].zero = true;
            if (nm && fused_norm) *fused_norm = true;
            done += k;
        }
        if (prolong && L.zero) CHK(op_prolong_add(c, l));   // unreachable in practice
        return MGX_OK;
    }
    if (prolong) CHK(op_prolong_add(c, l));
    for (int k = 0; k < sweeps; ++k) {
        if (c->opt.smoother == 2) {
            const bool z = L.zero;
            CHK(launch(c, MGX_K_GS, l, 40.0 * L.M(), [&] {
                mgx::launch_gs_sweep(L.u[L.cur], L.u[L.nxt()], L.rhs, L.v1, L.v2, L.n, L.pitch,
                                     L.coef, z, c->stream);
            }));
            L.cur = L.nxt();
            L.zero = false;
        } else {
            CHK(materialize(c, l));
            CHK(launch(c, MGX_K_GS, l, 40.0 * L.M(), [&] {
                mgx::launch_gs_colour(L.U(), L.rhs, L.v1, L.v2, L.n, L.pitch, L.coef, 0,
                                      c->stream);
                mgx::launch_gs_colour(L.U(), L.rhs, L.v1, L.v2, L.n, L.pitch, L.coef, 1,
                                      c->stream);
            }));
        }
    }
    if (restrict_) CHK(op_restrict(c, l));
    return MGX_OK;
}

int op_gs(mgx_ctx *c, int l, int sweeps) {
    return op_smooth(c, l, sweeps, false, false, false, nullptr);
}

// residual + compute_norm on level l, norm read back to the host (the one
// host sync per cycle, gs.cpp:86 / multigrid.cpp:105,113).
int read_norm(mgx_ctx *c, double *norm) {
    HIPCHK(hipMemcpyAsync(c->hscal, c->dscal, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    *norm = c->hscal[0];
    return MGX_OK;
}

int op_residual_norm(mgx_ctx *c, int l, double *norm, double bytes_per_pt) {
    CHK(materialize(c, l));
    Level &L = c->lv[l];
    CHK(launch(c, MGX_K_RESNORM, l, bytes_per_pt * L.M(), 32.0 * L.M(), [&] {
        mgx::launch_residual_norm(L.U(), L.rhs, L.v1, L.v2, L.n, L.pitch, L.coef, c->partials,
                                  c->dscal, c->stream);
    }));
    return read_norm(c, norm);
}

// residual -> restriction into rhs[l+1]; u[l+1] = 0 (multigrid.cpp:73-77).
int op_restrict(mgx_ctx *c, int l) {
    CHK(materialize(c, l));
    Level &F = c->lv[l], &C = c->lv[l + 1];
    CHK(launch(c, MGX_K_RESTRICT, l, 40.0 * F.M() + 24.0 * C.M(), 32.0 * F.M() + 8.0 * C.M(), [&] {
        mgx::launch_residual_restrict(F.U(), F.rhs, F.v1, F.v2, F.n, F.pitch, F.coef, C.rhs,
                                      C.pitch, c->stream);
    }));
    C.zero = true;
    return MGX_OK;
}

// u[l] += prolongation(u[l+1]) (multigrid.cpp:81-83).
int op_prolong_add(mgx_ctx *c, int l) {
    CHK(flush_coarse(c));   // a deferred coarsest solve must run before it is prolonged
    CHK(materialize(c, l));
    CHK(materialize(c, l + 1));
    Level &F = c->lv[l], &C = c->lv[l + 1];
    CHK(launch(c, MGX_K_PROLONG, l, 32.0 * F.M() + 8.0 * C.M(), 16.0 * F.M() + 8.0 * C.M(), [&] {
        mgx::launch_prolong_add(F.U(), F.pitch, C.U(), C.pitch, C.n, c->stream);
    }));
    return MGX_OK;
}

// A W-cycle's post-smoothing of visit sh and pre-smoothing of visit sh+1 on
// level l as one tile pass (launch_smooth_wpair): prolongation + add,
// 2 nsmooth sweeps, residual restricted into rhs[l+1], u[l+1] = 0 -- bitwise
// the two passes.  *done = false (nothing launched) where it does not apply.
long g_wpair = 1;   // tuning key "wpair"
int op_wpair(mgx_ctx *c, int l, bool *done) {
    *done = false;
    Level &L = c->lv[l], &Cl = c->lv[l + 1];
    const int k = c->opt.nsmooth;
    if (!g_wpair || c->opt.smoother != 0 || k < 1 || k > 3 || c->opt.fuse < k || L.zero)
        return MGX_OK;
    // The coarsest solve pending, fused: its workgroups read Cl.rhs at their
    // start while the pass's restriction stores the next visit's rhs, so that
    // goes to the level's second rhs buffer (swapped in after the launch);
    // without one the solve runs on its own first.
    if (c->cf_level == l + 1 && !Cl.rhs_alt) CHK(flush_coarse(c));
    const bool cfuse = c->cf_level == l + 1;
    if (Cl.zero && !cfuse) return MGX_OK;
    mgx::SmoothArgs A{};
    A.uin = L.u[L.cur];
    A.uout = L.u[L.nxt()];
    A.rhs = L.rhs;
    A.v1 = L.v1;
    A.v2 = L.v2;
    A.n = L.n;
    A.pitch = L.pitch;
    A.c = L.coef;
    A.uc = Cl.U();
    A.rhsc = cfuse ? Cl.rhs_alt : Cl.rhs;
    A.pitchc = Cl.pitch;
    A.partials = c->partials;
    A.norm_out = c->dscal;
    if (cfuse) take_coarse(c, l, A);
    CHK(check_coarse_rhs(A, mgx::kModeProlong | mgx::kModeRestrict));
    // post (prolong + add, k sweeps) + pre (k sweeps, restrict)
    const double bytes = (32.0 + 40.0 * k) * L.M() + 8.0 * Cl.M() + (40.0 * k + 40.0) * L.M() +
                         24.0 * Cl.M();
    const double cbytes = 8.0 * (3.0 * L.M() + 2.0 * L.Mv() + 2.0 * Cl.M());
    int blocks = 0;
    const size_t before = c->pending.size();
    CHK(launch(c, MGX_K_PSMOOTH, l, bytes, cbytes,
               [&] { blocks = mgx::launch_smooth_wpair(A, k, c->stream); }));
    if (blocks < 0) unlaunch(c, before);   // nothing launched
    if (blocks == -4) return flush_coarse(c);   // the two passes
    if (blocks < 0) return MGX_OK;   // a march level: the two passes as usual
    if (cfuse) {
        took_coarse(c, l);
        std::swap(Cl.rhs, Cl.rhs_alt);   // the restricted rhs is the current one
    }
    L.cur = L.nxt();
    Cl.zero = true;
    *done = true;
    return MGX_OK;
}

// Coarsest level: GS until |r| <= coarse_tol or coarse_maxit (multigrid.cpp:55-65),
// `reps` times in a row (a W-cycle's `shape` visits, multigrid.cpp:52): one
// launch for all of them when the level fits one workgroup.
int op_coarse(mgx_ctx *c, int l, int reps) {
    Level &L = c->lv[l];
    if (L.n <= mgx::kCoarseOneWgMaxN) {
        const bool z = L.zero;
        CHK(launch(c, MGX_K_COARSE, l, 88.0 * L.M() * reps, 40.0 * L.M(), [&] {
            mgx::launch_coarse_solve(L.U(), L.rhs, L.v1, L.v2, L.n, L.pitch, L.coef,
                                     c->opt.coarse_tol, c->opt.coarse_maxit, z, c->dscal + 2,
                                     c->stream, reps);
        }));
        L.zero = false;
        return MGX_OK;
    }
    for (int r = 0; r < reps; ++r) {
        int it = 0;
        double res = 1.0;
        while (it < c->opt.coarse_maxit && res > c->opt.coarse_tol) {
            bool fused = false;
            CHK(op_smooth(c, l, 1, false, false, true, &fused));
            if (fused)
                CHK(read_norm(c, &res));
            else
                CHK(op_residual_norm(c, l, &res, 48.0));
            ++it;
        }
        c->hscal[4] += it;
    }
    return MGX_OK;
}

long g_step_fuse = 1;   // tuning key "step_fuse"

// Can level 0 run the cross-cycle pass (post of cycle k + pre of cycle k+1)?
static bool cross_ok(mgx_ctx *c) {
    const Level &L = c->lv[0];
    return cross_cycle_on() && !c->dist && c->L > 1 && L.u[2] && c->opt.smoother == 0 &&
           c->opt.shape >= 1 && (c->opt.nsmooth == 2 || c->opt.nsmooth == 3) &&
           c->opt.fuse >= c->opt.nsmooth;
}

// The speculative next-cycle state is only valid while nothing but V-cycles
// touches the levels; every other mutating entry point drops it.
void drop_spec(mgx_ctx *c) {
    if (!c->lv.empty()) c->lv[0].spec = -1;
    c->step_spec = false;
}

// k_xsmooth on level 0: u_post (cycle k, returned by mg_outer if it stops
// here) into one free buffer, u_pre (cycle k+1's pre-smoothing) into the
// other, the residual of u_post -> c->dscal[0], the restriction of u_pre's
// residual -> rhs[1] (u[1] flagged zero for cycle k+1).
static int op_cross(mgx_ctx *c, bool store_post, bool rs = false) {
    Level &L = c->lv[0], &Cl = c->lv[1];
    CHK(materialize(c, 1));
    if (rs && !L.rhs_alt) return fail(MGX_E_INTERNAL, "step-mode cross pass without rhs_alt");
    int P = -1, Q = -1;
    for (int i = 0; i < 3; ++i)
        if (i != L.cur) (P < 0 ? P : Q) = i;
    mgx::XArgs A;
    A.uin = L.U();
    A.upost = L.u[P];
    A.upre = L.u[Q];
    A.rhs = L.rhs;
    A.v1 = L.v1;
    A.v2 = L.v2;
    A.uc = Cl.U();
    A.pitchc = Cl.pitch;
    A.rhsc = Cl.rhs;
    A.partials = c->partials;
    A.norm_out = c->dscal;
    A.n = L.n;
    A.pitch = L.pitch;
    A.c = L.coef;
    A.store_post = store_post;
    A.sa1 = L.sa1;
    A.sb1 = L.sb1;
    A.sa2 = L.sa2;
    A.sb2 = L.sb2;
    if (rs) {
        A.rhs_next = L.rhs_alt;
        A.norm2_out = c->dscal + 6;
    }
    const int k = c->opt.nsmooth;
    // algorithmic bytes: prolong+add, k sweeps, residual+norm (post of cycle
    // k) + k sweeps, residual+restriction (pre of cycle k+1), SURVEY 8d
    const double bytes = (32.0 + 40.0 * k + 48.0) * L.M() + 8.0 * Cl.M() +
                         (40.0 * k + 40.0) * L.M() + 24.0 * Cl.M();
    // compulsory: u, rhs, v1, v2 and the coarse u read once; u_pre (+ u_post)
    // and the coarse rhs written once
    // (step mode: + compute_rhs and the initial residual norm of the next
    // step, and its rhs written)
    // (with velocity factors v1 / v2 are not read: two fine arrays fewer)
    const double bytes_rs = rs ? (32.0 + 48.0) * L.M() : 0.0;
    const double cbytes = 8.0 * ((store_post ? 6.0 : 5.0) * L.M() - (L.sa1 ? 2.0 * L.M() : 0.0) +
                                 2.0 * Cl.M() + (rs ? L.M() : 0.0));
    int blocks = 0;
    CHK(launch(c, MGX_K_XSMOOTH, 0, bytes + bytes_rs, cbytes,
               [&] { blocks = mgx::launch_xsmooth(A, k, c->stream); }));
    if (blocks < 0) return fail(MGX_E_ARG, "launch_xsmooth: unsupported sweeps / mode");
    L.xin = L.cur;
    L.cur = P;
    L.spec = Q;
    L.zero = false;
    Cl.zero = true;
    return MGX_OK;
}

// mg_inner (multigrid.cpp:17-92).  If norm != nullptr (finest level only) the
// residual norm after the cycle (multigrid.cpp:112-113) is produced too, fused
// into the last post-smoothing pass when possible.
//
// Finest level with a norm (mg_outer's cycles): the post-smoothing of this
// cycle and the pre-smoothing of the NEXT one are one k_xsmooth pass, so a
// cycle is [pre (first cycle only) | coarse levels | cross pass]; a cycle that
// follows one starts from the speculative state the cross pass left.
// W-cycles (shape 2, multigrid.cpp:52): visit sh's post-smoothing of level 0
// and visit sh+1's pre-smoothing + restriction are adjacent too, so they are
// one cross pass as well (its u_post and norm unused): [pre | coarse | cross |
// coarse | cross] per W-cycle instead of four level-0 passes.
// tuning key "graph_level": > 0 = op_vcycle(c, graph_level) -- the whole
// sub-cycle of the small levels below a level: their tile / march passes and
// the coarsest solve -- is captured once per entry state as a hipGraph
// (hipStreamBeginCapture on the context's own stream) and replayed, one
// hipGraphLaunch instead of ~10 (V) or ~1000 (W) kernel launches; 0 (default)
// = launched one by one.  The round-6 kernel trace has no idle time between
// the launches of a cycle (profiles/r6_gaps_*.txt), so this only moves host
// work.  Not with per-launch profiling (prof 1; prof 2 times level 0 only),
// partitioned contexts or a borrowed stream, nor
// where the coarsest solve loops on the host (n > kCoarseOneWgMaxN).
long g_graph_level = 0;
long g_tuning_epoch = 0;   // bumped by every mgx_set_tuning: graphs of older settings are stale
long g_graph_captures = 0, g_graph_replays = 0;   // (read-only keys, for the tests)

// The host state a sub-cycle from level l reads and changes: per level its
// current u buffer, zero flag and rhs buffers, the deferred coarsest solve,
// and the process tuning epoch.  Equal keys = the same launches on the same
// buffers (everything else the passes read is fixed at creation / upload).
static std::vector<long> graph_state(const mgx_ctx *c, int l) {
    std::vector<long> k;
    for (int i = l; i < c->L; ++i) {
        const Level &L = c->lv[i];
        k.push_back(L.cur);
        k.push_back(L.zero ? 1 : 0);
        k.push_back((long)(uintptr_t)L.rhs);
        k.push_back((long)(uintptr_t)L.rhs_alt);
    }
    k.push_back(c->cf_level);
    k.push_back(c->cf_reps);
    k.push_back(g_tuning_epoch);
    return k;
}
static void set_graph_state(mgx_ctx *c, int l, const std::vector<long> &k) {
    size_t j = 0;
    for (int i = l; i < c->L; ++i) {
        Level &L = c->lv[i];
        L.cur = (int)k[j++];
        L.zero = k[j++] != 0;
        L.rhs = (double *)(uintptr_t)k[j++];
        L.rhs_alt = (double *)(uintptr_t)k[j++];
    }
    c->cf_level = (int)k[j++];
    c->cf_reps = (int)k[j++];
}
static bool graphable(const mgx_ctx *c, int l) {
    return g_graph_level > 0 && l == g_graph_level && !c->capturing && !c->dist &&
           c->own_stream && c->prof != 1 && c->opt.smoother == 0 && l >= 1 && l < c->L - 1 &&
           c->lv[c->L - 1].n <= mgx::kCoarseOneWgMaxN;
}
void free_graphs(mgx_ctx *c) {
    for (auto &g : c->graphs)
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
    c->graphs.clear();
}
static int graph_vcycle(mgx_ctx *c, int l) {
    const std::vector<long> key = graph_state(c, l);
    for (auto &g : c->graphs)
        if (g.key == key) {
            HIPCHK(hipGraphLaunch(g.exec, c->stream));
            set_graph_state(c, l, g.end);
            ++g_graph_replays;
            return MGX_OK;
        }
    if (c->graphs.size() >= 8) free_graphs(c);   // (stale entry states: start over)
    HIPCHK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    c->capturing = true;
    const int rc = op_vcycle(c, l);
    c->capturing = false;
    hipGraph_t graph = nullptr;
    const hipError_t e = hipStreamEndCapture(c->stream, &graph);
    if (rc != MGX_OK) {
        if (graph) (void)hipGraphDestroy(graph);
        return rc;
    }
    if (e != hipSuccess) return fail(MGX_E_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
    mgx_ctx::Graph g;
    g.key = key;
    g.end = graph_state(c, l);
    const hipError_t ei = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (ei != hipSuccess) return fail(MGX_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
    c->graphs.push_back(g);
    ++g_graph_captures;
    // (the capture only recorded the launches: run them now)
    HIPCHK(hipGraphLaunch(g.exec, c->stream));
    return MGX_OK;
}

int op_vcycle(mgx_ctx *c, int l, double *norm, bool store_post) {
    if (!norm && graphable(c, l)) return graph_vcycle(c, l);
    if (l == 0 && norm && cross_ok(c)) {
        Level &L = c->lv[0];
        if (L.spec >= 0) {   // pre-smoothing + restriction already done
            L.cur = L.spec;
            L.spec = -1;
        } else {
            CHK(op_smooth(c, 0, c->opt.nsmooth, false, /*restrict=*/true, false, nullptr));
        }
        for (int sh = 1; sh < c->opt.shape; ++sh) {
            CHK(op_vcycle(c, 1));
            CHK(op_cross(c, /*store_post=*/false));
            L.cur = L.spec;   // visit sh+1 starts from the pass's u_pre
            L.spec = -1;
        }
        CHK(op_vcycle(c, 1));
        if (c->post_only && c->step_next && mgx::xstep_supported(L.n) && L.coef.dgs > 0) {
            // the last cycle of a time step whose next step follows: the cross
            // pass in step mode (u_post stored; B pre-smooths the next step)
            CHK(op_cross(c, /*store_post=*/true, /*rs=*/true));
            HIPCHK(hipMemcpyAsync(c->hscal, c->dscal, sizeof(double), hipMemcpyDeviceToHost,
                                  c->stream));
            HIPCHK(hipMemcpyAsync(c->hscal + 6, c->dscal + 6, sizeof(double),
                                  hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            *norm = c->hscal[0];
            c->step_res0 = c->hscal[6];
            c->step_spec = true;
            return MGX_OK;
        }
        if (c->post_only) {   // the last cycle: prolongation + post-smoothing + norm only
            bool fused = false;
            CHK(op_smooth(c, 0, c->opt.nsmooth, /*prolong=*/true, false, /*norm=*/true, &fused));
            L.spec = -1;
            return fused ? read_norm(c, norm) : op_residual_norm(c, 0, norm);
        }
        CHK(op_cross(c, store_post));
        return read_norm(c, norm);
    }
    if (l == 0) drop_spec(c);
    bool have_norm = false;
    bool pre_done = false;   // visit sh's pre-smoothing ran fused with sh-1's post
    // (the coarsest level's `shape` solves in a row: one op_coarse)
    for (int sh = 0; sh < (l == c->L - 1 ? 1 : c->opt.shape); ++sh) {
        const bool last = sh == c->opt.shape - 1;
        if (l == c->L - 1) {
            if (coarse_fusable(c, l)) {   // taken by the next prolongation pass
                c->cf_level = l;
                c->cf_reps = c->opt.shape;
            } else {
                CHK(op_coarse(c, l, c->opt.shape));
            }
        } else {
            if (!pre_done)
                CHK(op_smooth(c, l, c->opt.nsmooth, false, /*restrict=*/true, false, nullptr));
            pre_done = false;
            CHK(op_vcycle(c, l + 1));
            // W-cycles: this visit's post- and the next visit's pre-smoothing
            // back to back -- one tile pass where the level runs as tiles
            if (!last) {
                bool fused = false;
                CHK(op_wpair(c, l, &fused));
                if (fused) {
                    pre_done = true;
                    continue;
                }
            }
            CHK(op_smooth(c, l, c->opt.nsmooth, /*prolong=*/true, false, norm && last,
                          &have_norm));
            CHK(flush_coarse(c));   // (taken above; never left pending)
        }
    }
    if (norm) {
        if (have_norm)
            CHK(read_norm(c, norm));
        else
            CHK(op_residual_norm(c, l, norm));
    }
    return MGX_OK;
}

int op_rhs(mgx_ctx *c) {
    drop_spec(c);
    CHK(materialize(c, 0));
    Level &L = c->lv[0];
    return launch(c, MGX_K_RHS, 0, 32.0 * L.M(), [&] {
        mgx::launch_rhs(L.rhs, L.U(), L.v1, L.v2, L.n, L.pitch, L.coef, c->stream);
    });
}

// compute_rhs (gs.cpp:24) + mg_outer's initial residual norm (multigrid.cpp:104)
// in one pass over u, v1, v2 (a time step's first two reads of the fields)
static int op_rhs_norm(mgx_ctx *c, double *res0) {
    drop_spec(c);
    CHK(materialize(c, 0));
    Level &L = c->lv[0];
    CHK(launch(c, MGX_K_RHS, 0, 32.0 * L.M() + 48.0 * L.M(), 32.0 * L.M(), [&] {
        mgx::launch_rhs_norm(L.rhs, L.U(), L.v1, L.v2, L.n, L.pitch, L.coef, c->partials,
                             c->dscal, c->stream);
    }));
    return read_norm(c, res0);
}

// A time step's compute_rhs, mg_outer's initial norm AND the first cycle's
// pre-smoothing + restriction in ONE pass over u, v1, v2 (k_wsmooth mode
// kModeRhsNorm): u_pre goes to the free buffer and is left as the
// speculative state the first cycle starts from (Level::spec, as after a
// cross pass).  Only where the cross-cycle schedule runs (so the first cycle
// takes that state) and level 0 is a row march.  -> false: not applicable.
static bool step_fusable(mgx_ctx *c) {
    return cross_ok(c) && c->lv[0].n > mgx::get_tile_max_n() && g_step_fuse != 0;
}
static int op_rhs_norm_pre(mgx_ctx *c, double *res0) {
    drop_spec(c);
    CHK(materialize(c, 0));
    CHK(materialize(c, 1));
    Level &L = c->lv[0], &Cl = c->lv[1];
    const int k = c->opt.nsmooth;
    const int out = L.nxt();
    mgx::SmoothArgs A{};
    A.uin = L.u[L.cur];
    A.uout = L.u[out];
    A.rhs = L.rhs;
    A.rhs_out = L.rhs;
    A.v1 = L.v1;
    A.v2 = L.v2;
    A.n = L.n;
    A.pitch = L.pitch;
    A.c = L.coef;
    A.uc = Cl.U();
    A.rhsc = Cl.rhs;
    A.pitchc = Cl.pitch;
    A.partials = c->partials;
    A.norm_out = c->dscal;
    // algorithmic: compute_rhs 32, residual+norm 48, k sweeps 40 each,
    // residual+restriction 40 + 24 per coarse point; compulsory: u, v1, v2
    // read, rhs and u_pre written, the coarse rhs written
    const double bytes = (32.0 + 48.0 + 40.0 * k + 40.0) * L.M() + 24.0 * Cl.M();
    const double cbytes = 8.0 * (5.0 * L.M() + Cl.M());
    int blocks = 0;
    CHK(launch(c, MGX_K_RHS, 0, bytes, cbytes, [&] {
        blocks = mgx::launch_smooth(A, k, mgx::kModeRestrict | mgx::kModeRhsNorm, c->stream);
    }));
    if (blocks < 0) return fail(MGX_E_ARG, "launch_smooth: rhs+norm+pre-smoothing unsupported");
    L.spec = out;   // the first cycle's pre-smoothed u (op_vcycle takes it)
    L.zero = false;
    Cl.zero = true;
    return read_norm(c, res0);
}

// mg_outer (multigrid.cpp:97-120).
// one V-cycle + the residual norm after it, single GPU or partitioned
// store_post = false: the caller runs another cycle right away, so this
// cycle's solution is never observed (only its norm); skip writing it
int cycle_norm(mgx_ctx *c, double *res, bool store_post = true) {
    if (c->dist) return dist_vcycle(c, res, store_post);
    return op_vcycle(c, 0, res, store_post);
}
int norm0(mgx_ctx *c, double *res) {
    if (c->dist) return dist_residual_norm(c, res);
    return op_residual_norm(c, 0, res);
}

// have_res0: the caller computed the initial norm (fused with compute_rhs)
// The cycle that converged did not store its u_post (predicted to go on):
// recompute it from the cycle's input and the level-1 correction, both still
// intact -- the post-smoothing pass alone, bitwise the cross pass's u_post
// (the same prolongation and sweeps: tests/test_gpu_cross.py).
static int op_redo_post(mgx_ctx *c) {
    Level &L = c->lv[0];
    if (L.xin < 0) return fail(MGX_E_INTERNAL, "redo post-smoothing: no cross pass input");
    L.cur = L.xin;
    L.spec = -1;
    L.zero = false;
    c->lv[1].zero = false;   // u[1] still holds the correction the pass prolonged
    return op_smooth(c, 0, c->opt.nsmooth, /*prolong=*/true, false, false, nullptr);
}

// op_vcycle / dist_vcycle with a norm would run the cross-cycle pass
static bool post_predictable(mgx_ctx *c) {
    if (!c->dist) return cross_ok(c);
    if (dist_la(c) == 0) return cross_ok(dist_sub(c, 0));   // everything replicated
    return dist_post_predictable(c);
}
static int redo_post(mgx_ctx *c) {
    if (!c->dist) return op_redo_post(c);
    if (dist_la(c) == 0) {
        for (int i = 0; i < dist_nsub(c); ++i) CHK(op_redo_post(dist_sub(c, i)));
        return MGX_OK;
    }
    return dist_redo_post(c);
}

static void set_post_only(mgx_ctx *c, bool v) {
    c->post_only = v;
    if (c->dist)
        for (int i = 0; i < dist_nsub(c); ++i) dist_sub(c, i)->post_only = v;
}

// tuning key "post_only": a cycle whose extrapolated norm is within tol /
// post_only (or the last cycle mg_outer may run) skips the next cycle's
// pre-smoothing: its finest level runs the post-smoothing pass alone, not the
// cross pass (2.7 GB of u_pre + coarse rhs writes and B's sweeps saved); if it
// does not converge after all, the next cycle pre-smooths from its u_post
// (0 = never; -1 = every cycle, the test of that path)
long g_post_only = 10;

// tuning key "post_predict": mg_outer stores a cycle's u_post only when the
// cycle is predicted to converge -- its norm extrapolated with the last
// reduction factor within post_predict x tol -- and recomputes it in the
// rare case a cycle converges unannounced (0 = always store; -1 = never
// store, always recompute: the test of the recompute path)
double g_post_predict = 10.0;

int op_mg_outer(mgx_ctx *c, double tol, int *cycles, double *res0_out, double *res_out,
                const double *have_res0 = nullptr) {
    double res0 = 0, res = 0;
    if (have_res0)
        res0 = *have_res0;
    else
        CHK(norm0(c, &res0));
    res = res0;
    int iter = 0;
    // the u_post of a cycle that does not converge is never observed: the
    // cross pass skips storing it (2.15 GB at N=16384) when so predicted
    const bool predict = g_post_predict != 0 && post_predictable(c);
    double prev = res0;
    for (; iter < c->opt.max_cycle && res / res0 > tol; ++iter) {
        bool store = true, last = false;
        if (predict) {
            const double pred = res * (res / prev);
            if (iter + 1 < c->opt.max_cycle)   // the last allowed cycle always stores
                store = g_post_predict > 0 && pred <= g_post_predict * tol * res0;
            last = g_post_only < 0 ||
                   (g_post_only > 0 && (iter + 1 == c->opt.max_cycle ||
                                        pred * (double)g_post_only <= tol * res0));
        }
        prev = res;
        set_post_only(c, last);
        const int rc = cycle_norm(c, &res, store);
        set_post_only(c, false);
        CHK(rc);
        if (c->step_spec && res / res0 > tol) {
            // step mode, but the cycle did not converge: its pre-smoothing was
            // the next step's (other rhs); the next cycle pre-smooths from u_post
            c->step_spec = false;
            c->lv[0].spec = -1;
        }
        if (!store && !last && !(res / res0 > tol)) CHK(redo_post(c));
    }
    if (cycles) *cycles = iter;
    if (res0_out) *res0_out = res0;
    if (res_out) *res_out = res;
    if (iter == c->opt.max_cycle) return fail(MGX_E_NOCONV, "mg_outer did not converge");
    return MGX_OK;
}

// Coarse velocity tower (multigrid.cpp:148-160).  Reference mode reproduces
// the reference's index arithmetic on flat (n/2+1)^2 buffers, zero filled
// (SURVEY K2); correct mode injects every level from the one above.
int build_tower(mgx_ctx *c) {
    const long N = c->N;
    for (int f = 0; f < 2; ++f) {
        double *fine = f == 0 ? c->lv[0].v1 : c->lv[0].v2;
        if (c->opt.tower_mode == MGX_TOWER_CORRECT) {
            for (int l = 1; l < c->L; ++l) {
                Level &A = c->lv[l - 1], &B = c->lv[l];
                const double *src = f == 0 ? A.v1 : A.v2;
                double *dst = f == 0 ? B.v1 : B.v2;
                mgx::launch_injection(dst, B.pitch, src, A.pitch, B.n + 1, c->stream);
                CHK(check_launch("injection"));
            }
            continue;
        }
        if (c->L < 2) continue;
        // flat level-0 copy of the fine field in the reference layout
        HIPCHK(hipMemcpy2DAsync(c->stage[0], (N + 1) * sizeof(double), fine,
                                c->lv[0].pitch * sizeof(double), (N + 1) * sizeof(double), N + 1,
                                hipMemcpyDeviceToDevice, c->stream));
        const long ni = (N >> 1) + 1;   // multigrid.cpp:150
        for (int l = 1; l < c->L; ++l) {
            double *prev = c->stage[(l - 1) & 1], *next = c->stage[l & 1];
            HIPCHK(hipMemsetAsync(next, 0, sizeof(double) * ni * ni, c->stream));
            // restriction(vtow[l], vtow[l-1], ni-1): next[I*(ni/2... )] per gs.cpp:283
            const long nr = ni - 1;   // the "n" passed to restriction
            mgx::launch_injection(next, nr / 2 + 1, prev, nr + 1, nr / 2 + 1, c->stream);
            CHK(check_launch("tower injection"));
            Level &B = c->lv[l];
            double *dst = f == 0 ? B.v1 : B.v2;
            // level l reads its buffer with its own width n_l+1 (multigrid.cpp:46-47)
            HIPCHK(hipMemcpy2DAsync(dst, B.pitch * sizeof(double), next,
                                    (B.n + 1) * sizeof(double), (B.n + 1) * sizeof(double),
                                    B.n + 1, hipMemcpyDeviceToDevice, c->stream));
        }
    }
    return MGX_OK;
}

// tuning key "zero_rows": 1 (default) = find_zero_rows at upload; 0 = read
// every velocity row from HBM
long g_zero_rows = 1;

int find_zero_rows(mgx_ctx *c) {
    for (auto &L : c->lv) L.vz = 0x7fffffff;
    if (c->L < 2 || !g_zero_rows) return MGX_OK;
    int *dflags = nullptr;
    const long nmax = c->lv[1].n + 1;
    HIPCHK(hipMalloc(&dflags, sizeof(int) * 2 * nmax));
    std::vector<int> h(2 * nmax);
    int rc = MGX_OK;
    for (int l = 1; l < c->L && rc == MGX_OK; ++l) {
        Level &L = c->lv[l];
        mgx::launch_row_nonzero(L.v1, L.pitch, L.n, dflags, c->stream);
        mgx::launch_row_nonzero(L.v2, L.pitch, L.n, dflags + nmax, c->stream);
        if (check_launch("row_nonzero") != MGX_OK ||
            hipMemcpyAsync(h.data(), dflags, sizeof(int) * 2 * nmax, hipMemcpyDeviceToHost,
                           c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess) {
            rc = fail(MGX_E_HIP, "find_zero_rows");
            break;
        }
        long last = -1;
        for (long i = 0; i <= L.n; ++i)
            if (h[i] || h[nmax + i]) last = i;
        L.vz = (int)(last + 1);
    }
    (void)hipFree(dflags);
    return rc;
}

// The coarse levels that generate their velocity (Level::vgen): levels 1-2 of
// the reference tower (the injection quirk's closed form) or every level of
// the correct tower (strided: the finest factors at rows / columns 2^l i,
// 2^l j), below the coarsest (whose solve reads the arrays), when the finest
// factors exist and every entry of the level equals the generator's bits
// (k_vgen_check).  a1, a2: the finest row factors.
int find_vgen(mgx_ctx *c, const std::vector<double> &a1, const std::vector<double> &a2) {
    for (auto &L : c->lv) L.vgen = false;
    (void)hipFree(c->vga);
    c->vga = nullptr;
    const Level &F = c->lv[0];
    const bool strided = c->opt.tower_mode == MGX_TOWER_CORRECT;
    // (the reference closed form's integer products fit in int up to N = 2^15)
    if (!F.sa1 || c->L < 3 || (c->N & 3) || (!strided && c->N > 32768) ||
        (long)a1.size() != c->N + 1 || (long)a2.size() != c->N + 1)
        return MGX_OK;
    std::vector<double2> h((size_t)c->N + 2, make_double2(0.0, 0.0));
    for (long I = 0; I <= c->N; ++I) h[(size_t)I] = make_double2(a1[(size_t)I], a2[(size_t)I]);
    HIPCHK(hipMalloc(&c->vga, sizeof(double2) * h.size()));
    const int top = strided ? c->L - 2 : std::min(c->L - 2, 2);
    std::vector<int> ok(c->L, 0), one(c->L, 1);
    int *dok = nullptr;
    HIPCHK(hipMalloc(&dok, sizeof(int) * c->L));
    int rc = MGX_OK;
    if (hipMemcpyAsync(c->vga, h.data(), sizeof(double2) * h.size(), hipMemcpyHostToDevice,
                       c->stream) != hipSuccess ||
        hipMemcpyAsync(dok, one.data(), sizeof(int) * c->L, hipMemcpyHostToDevice, c->stream) !=
            hipSuccess)
        rc = fail(MGX_E_HIP, "find_vgen");
    for (int l = 1; l <= top && rc == MGX_OK; ++l) {
        const Level &L = c->lv[l];
        if ((L.n << l) != c->N || (L.n & 1)) continue;
        mgx::launch_vgen_check(L.v1, L.v2, L.n, L.pitch, level_vgen(c, l), dok + l, c->stream);
        rc = check_launch("vgen_check");
    }
    if (rc == MGX_OK &&
        (hipMemcpyAsync(ok.data(), dok, sizeof(int) * c->L, hipMemcpyDeviceToHost, c->stream) !=
             hipSuccess ||
         hipStreamSynchronize(c->stream) != hipSuccess))
        rc = fail(MGX_E_HIP, "find_vgen");
    (void)hipFree(dok);
    bool any = false;
    for (int l = 1; l <= top && rc == MGX_OK; ++l) {
        Level &L = c->lv[l];
        L.vgen = (L.n << l) == c->N && !(L.n & 1) && ok[l] == 1;
        any = any || L.vgen;
    }
    if (!any) {
        (void)hipFree(c->vga);
        c->vga = nullptr;
    }
    return rc;
}

void free_ctx(mgx_ctx *c) {
    if (!c) return;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->dist) dist_free(c);
    for (auto &L : c->lv) {
        (void)hipFree(L.u[0]);
        (void)hipFree(L.u[1]);
        (void)hipFree(L.u[2]);
        (void)hipFree(L.rhs);
        (void)hipFree(L.rhs_alt);
        (void)hipFree(L.v1);
        (void)hipFree(L.v2);
        free_level_factors(L);
    }
    (void)hipFree(c->partials);
    (void)hipFree(c->dscal);
    (void)hipFree(c->stage[0]);
    (void)hipFree(c->stage[1]);
    (void)hipFree(c->zrow);
    (void)hipFree(c->vga);
    if (c->hscal) (void)hipHostFree(c->hscal);
    for (auto &r : c->pending) {
        (void)hipEventDestroy(r.e0);
        (void)hipEventDestroy(r.e1);
    }
    for (auto e : c->pool) (void)hipEventDestroy(e);
    free_graphs(c);
    if (c->stream && c->own_stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

bool is_pow2(long n) { return n >= 2 && (n & (n - 1)) == 0; }

// raw-op scratch (norm partials + result), shared by the gs.h-mirror entry points
std::mutex g_raw_mu;
double *g_raw_scratch = nullptr;
int g_raw_dev = -1;

int raw_scratch(double **p) {
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    if (!g_raw_scratch || g_raw_dev != dev) {
        HIPCHK(hipMalloc(&g_raw_scratch, sizeof(double) * (mgx::norm_partials_size() + 8)));
        g_raw_dev = dev;
    }
    *p = g_raw_scratch;
    return MGX_OK;
}

}  // namespace mgxi

using namespace mgxi;

// =================================================================== C ABI
extern "C" {

const char *mgx_last_error(void) { return g_err.c_str(); }
int mgx_version(void) { return 100; }

void mgx_default_options(mgx_options *o) {
    o->nsmooth = 3;          // multigrid.cpp:41
    o->shape = 1;            // multigrid.cpp:241
    o->tower_mode = MGX_TOWER_REFERENCE;
    o->device = -1;          // current device
    o->coarse_tol = 1e-5;    // multigrid.cpp:60
    o->coarse_maxit = 1000;  // multigrid.cpp:60
    o->max_cycle = 50;       // multigrid.cpp:94
    o->smoother = 0;
    o->fuse = 3;
    o->fp_mode = MGX_FP_BITWISE;
}

// ---- gs.h mirror (reference layout, device pointers, null stream)
int mgx_gauss_seidel(double *u, const double *rhs, long n, const double *v1, const double *v2,
                     double k, double nu, double h) {
    if (!u || !rhs || !v1 || !v2 || n < 2) return fail(MGX_E_ARG, "mgx_gauss_seidel: bad args");
    mgx::Coef c = mgx::make_coef(k, nu, h);
    mgx::launch_raw_gs_colour(u, rhs, v1, v2, n, c, 0, nullptr);
    mgx::launch_raw_gs_colour(u, rhs, v1, v2, n, c, 1, nullptr);
    return check_launch("mgx_gauss_seidel");
}
int mgx_residual(double *res, const double *u, const double *rhs, long n, const double *v1,
                 const double *v2, double k, double nu, double h) {
    if (!res || !u || !rhs || !v1 || !v2 || n < 2) return fail(MGX_E_ARG, "mgx_residual: bad args");
    mgx::launch_raw_residual(res, u, rhs, v1, v2, n, mgx::make_coef(k, nu, h), nullptr);
    return check_launch("mgx_residual");
}
int mgx_compute_norm(const double *res, long n, double *norm) {
    if (!res || !norm || n < 1) return fail(MGX_E_ARG, "mgx_compute_norm: bad args");
    std::lock_guard<std::mutex> g(g_raw_mu);
    double *s = nullptr;
    CHK(raw_scratch(&s));
    double *out = s + mgx::norm_partials_size();
    mgx::launch_norm(res, n, n + 1, s, out, nullptr);
    CHK(check_launch("mgx_compute_norm"));
    HIPCHK(hipMemcpy(norm, out, sizeof(double), hipMemcpyDeviceToHost));
    return MGX_OK;
}
int mgx_prolongation(double *up, const double *u, long n) {
    if (!up || !u || n < 1) return fail(MGX_E_ARG, "mgx_prolongation: bad args");
    mgx::launch_raw_prolongation(up, u, n, nullptr);
    return check_launch("mgx_prolongation");
}
int mgx_restriction(double *u, const double *up, long n) {
    if (!u || !up || n < 2) return fail(MGX_E_ARG, "mgx_restriction: bad args");
    mgx::launch_injection(u, n / 2 + 1, up, n + 1, n / 2 + 1, nullptr);
    return check_launch("mgx_restriction");
}
int mgx_compute_rhs(double *rhs, const double *u, long n, const double *v1, const double *v2,
                    double k, double nu, double h) {
    if (!rhs || !u || !v1 || !v2 || n < 2) return fail(MGX_E_ARG, "mgx_compute_rhs: bad args");
    mgx::launch_raw_rhs(rhs, u, v1, v2, n, mgx::make_coef(k, nu, h), nullptr);
    return check_launch("mgx_compute_rhs");
}

}  // extern "C"

// ---- context
int mgxi::create_ctx(mgx_ctx **out, long n, int maxlvl, double dt, double nu,
                     const mgx_options *opt, hipStream_t borrowed) {
    if (!out) return fail(MGX_E_ARG, "mgx_create: null out");
    *out = nullptr;
    if (!is_pow2(n)) return fail(MGX_E_ARG, "mgx_create: n must be a power of two >= 2");
    if (maxlvl < 1 || (n >> (maxlvl - 1)) < 2)
        return fail(MGX_E_ARG, "mgx_create: maxlvl must satisfy 1 <= maxlvl, n>>(maxlvl-1) >= 2");
    mgx_options o;
    mgx_default_options(&o);
    if (opt) o = *opt;
    if (o.fuse < 1 || o.fuse > mgx::kSmoothMaxSweeps) o.fuse = mgx::kSmoothMaxSweeps;
    if (o.nsmooth < 0 || o.shape < 1 || o.coarse_maxit < 1 || o.max_cycle < 1 ||
        o.smoother < 0 || o.smoother > 2 || (o.fp_mode != MGX_FP_BITWISE && o.fp_mode != MGX_FP_FMA))
        return fail(MGX_E_ARG, "mgx_create: bad options");
    mgx_ctx *c = new mgx_ctx();
    c->N = n;
    c->L = maxlvl;
    c->dt = dt;
    c->nu = nu;
    c->opt = o;
    auto bail = [&](int rc) {
        free_ctx(c);
        return rc;
    };
    if (o.device >= 0) {
        hipError_t e = hipSetDevice(o.device);
        if (e != hipSuccess) return bail(fail(MGX_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e)));
    }
    if (hipGetDevice(&c->device) != hipSuccess) return bail(fail(MGX_E_HIP, "hipGetDevice"));
    if (borrowed) {
        c->stream = borrowed;
        c->own_stream = false;
    } else if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        return bail(fail(MGX_E_HIP, "hipStreamCreate"));
    }
    c->lv.resize(maxlvl);
    double h = 1.0 / n;   // dx (multigrid.cpp:194), doubled per level (:49)
    for (int l = 0; l < maxlvl; ++l) {
        Level &L = c->lv[l];
        L.n = n >> l;
        L.pitch = mgx::tower_pitch(L.n);
        L.coef = mgx::make_coef(dt, nu, h, o.fp_mode == MGX_FP_FMA);
        h = 2 * h;
        const size_t bytes = sizeof(double) * L.pitch * (L.n + 1);
        double **bufs[5] = {&L.u[0], &L.u[1], &L.rhs, &L.v1, &L.v2};
        for (double **b : bufs) {
            if (hipMalloc(b, bytes) != hipSuccess)
                return bail(fail(MGX_E_HIP, "hipMalloc (level tower): out of device memory"));
            if (hipMemsetAsync(*b, 0, bytes, c->stream) != hipSuccess)
                return bail(fail(MGX_E_HIP, "hipMemset"));
        }
    }
    if (maxlvl >= 3 && c->lv[maxlvl - 1].n <= mgx::kCoarseLdsMaxN) {
        // coarsest level: the second rhs of a W-cycle pair pass with the fused
        // solve (op_wpair); zero boundary, as the restriction writes the interior
        Level &L = c->lv[maxlvl - 1];
        const size_t bytes = sizeof(double) * L.pitch * (L.n + 1);
        if (hipMalloc(&L.rhs_alt, bytes) != hipSuccess ||
            hipMemsetAsync(L.rhs_alt, 0, bytes, c->stream) != hipSuccess)
            return bail(fail(MGX_E_HIP, "hipMalloc (coarsest rhs)"));
    }
    if (maxlvl > 1 && n >= kCrossMinN) {   // third finest-level buffer: cross-cycle pass
        Level &L = c->lv[0];
        const size_t bytes = sizeof(double) * L.pitch * (L.n + 1);
        if (hipMalloc(&L.u[2], bytes) != hipSuccess)
            return bail(fail(MGX_E_HIP, "hipMalloc (level tower): out of device memory"));
    }
    const size_t flat = sizeof(double) * (n + 1) * (n + 1);
    // (two partial arrays: the cross pass's time-step mode sums two norms)
    if (hipMalloc(&c->zrow, sizeof(double) * c->lv[0].pitch) != hipSuccess ||
        hipMemsetAsync(c->zrow, 0, sizeof(double) * c->lv[0].pitch, c->stream) != hipSuccess)
        return bail(fail(MGX_E_HIP, "hipMalloc (zero row)"));
    if (hipMalloc(&c->partials, 2 * sizeof(double) * mgx::norm_partials_size()) != hipSuccess ||
        hipMalloc(&c->dscal, sizeof(double) * 8) != hipSuccess ||
        hipHostMalloc(&c->hscal, sizeof(double) * 8) != hipSuccess)
        return bail(fail(MGX_E_HIP, "hipMalloc (scratch)"));
    if (maxlvl > 1 && o.tower_mode == MGX_TOWER_REFERENCE) {
        if (hipMalloc(&c->stage[0], flat) != hipSuccess || hipMalloc(&c->stage[1], flat) != hipSuccess)
            return bail(fail(MGX_E_HIP, "hipMalloc (staging)"));
    }
    (void)hipMemsetAsync(c->dscal, 0, sizeof(double) * 8, c->stream);
    memset(c->hscal, 0, sizeof(double) * 8);
    if (hipStreamSynchronize(c->stream) != hipSuccess) return bail(fail(MGX_E_HIP, "sync"));
    *out = c;
    return MGX_OK;
}

extern "C" {

int mgx_create(mgx_ctx **out, long n, int maxlvl, double dt, double nu, const mgx_options *opt) {
    return create_ctx(out, n, maxlvl, dt, nu, opt, nullptr);
}

int mgx_destroy(mgx_ctx *c) {
    free_ctx(c);
    return MGX_OK;
}

}  // extern "C"

int mgxi::upload_ctx(mgx_ctx *c, const double *u0, const double *v1, const double *v2,
                     hipMemcpyKind kind) {
    if (!c || !u0 || !v1 || !v2) return fail(MGX_E_ARG, "mgx_upload: bad args");
    HIPCHK(hipSetDevice(c->device));
    Level &L = c->lv[0];
    const size_t row = (c->N + 1) * sizeof(double);
    L.cur = 0;
    L.zero = false;
    L.spec = -1;
    c->step_spec = false;   // a pending next-step state belongs to the old fields
    const double *src[3] = {u0, v1, v2};
    double *dst[3] = {L.u[0], L.v1, L.v2};
    for (int k = 0; k < 3; ++k)
        HIPCHK(hipMemcpy2DAsync(dst[k], L.pitch * sizeof(double), src[k], row, row, c->N + 1,
                                kind, c->stream));
    for (int l = 1; l < c->L; ++l) {
        c->lv[l].cur = 0;
        c->lv[l].zero = false;
    }
    CHK(build_tower(c));
    CHK(find_zero_rows(c));
    // exact velocity factors for the finest level's cross pass (host data only;
    // a device upload keeps the 2-D arrays)
    free_level_factors(L);
    std::vector<double> a1, b1, a2, b2;
    if (kind == hipMemcpyHostToDevice && c->L > 1 && c->N >= kCrossMinN &&
        factor_velocity(v1, v2, c->N, 0, c->N + 1, L.coef.h * 0.5, a1, b1, a2, b2))
        CHK(set_level_factors(L, 0, a1, b1, a2, b2, c->stream));
    CHK(find_vgen(c, a1, a2));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MGX_OK;
}

extern "C" {

int mgx_upload(mgx_ctx *c, const double *u0, const double *v1, const double *v2) {
    if (c && c->dist) return dist_upload(c, u0, v1, v2, hipMemcpyHostToDevice);
    return upload_ctx(c, u0, v1, v2, hipMemcpyHostToDevice);
}
int mgx_upload_device(mgx_ctx *c, const double *u0, const double *v1, const double *v2) {
    if (c && c->dist) return dist_upload(c, u0, v1, v2, hipMemcpyDeviceToDevice);
    return upload_ctx(c, u0, v1, v2, hipMemcpyDeviceToDevice);
}

static int download_impl(mgx_ctx *c, int level, int field, double *out, hipMemcpyKind kind) {
    if (!c || !out || level < 0 || level >= c->L || field < 0 || field > 3)
        return fail(MGX_E_ARG, "mgx_download: bad args");
    HIPCHK(hipSetDevice(c->device));
    CHK(materialize(c, level));
    Level &L = c->lv[level];
    const double *src = field == 0 ? L.U() : field == 1 ? L.rhs : field == 2 ? L.v1 : L.v2;
    const size_t row = (L.n + 1) * sizeof(double);
    HIPCHK(hipMemcpy2DAsync(out, row, src, L.pitch * sizeof(double), row, L.n + 1, kind,
                            c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MGX_OK;
}

int mgx_download(mgx_ctx *c, double *u) {
    if (c && c->dist) return dist_download(c, u, hipMemcpyDeviceToHost);
    return download_impl(c, 0, 0, u, hipMemcpyDeviceToHost);
}
int mgx_download_device(mgx_ctx *c, double *u) {
    if (c && c->dist) return dist_download(c, u, hipMemcpyDeviceToDevice);
    return download_impl(c, 0, 0, u, hipMemcpyDeviceToDevice);
}
int mgx_download_level(mgx_ctx *c, int level, int field, double *out) {
    if (c && c->dist) return fail(MGX_E_ARG, "mgx_download_level: not available on a partitioned context");
    return download_impl(c, level, field, out, hipMemcpyDeviceToHost);
}
int mgx_owned_rows(mgx_ctx *c, int part, int *ra, int *rb) {
    if (!c || !ra || !rb) return fail(MGX_E_ARG, "mgx_owned_rows: bad args");
    if (c->dist) return dist_owned_rows(c, part, ra, rb);
    if (part != 0) return fail(MGX_E_ARG, "mgx_owned_rows: a single-GPU context has part 0 only");
    *ra = 0;
    *rb = (int)c->N + 1;
    return MGX_OK;
}
int mgx_download_rows(mgx_ctx *c, int part, double *rows) {
    if (!c || !rows) return fail(MGX_E_ARG, "mgx_download_rows: bad args");
    if (c->dist) return dist_download_rows(c, part, rows, hipMemcpyDeviceToHost);
    if (part != 0) return fail(MGX_E_ARG, "mgx_download_rows: a single-GPU context has part 0 only");
    return download_impl(c, 0, 0, rows, hipMemcpyDeviceToHost);
}

static int no_dist(mgx_ctx *c, const char *what) {
    return fail(MGX_E_ARG, std::string(what) + ": per-level ops are not available on a "
                                               "partitioned context (use vcycle/mg_outer/step)");
}
int mgx_rhs(mgx_ctx *c) {
    if (!c) return fail(MGX_E_ARG, "null ctx");
    if (c->dist) return dist_rhs(c);
    return op_rhs(c);
}
int mgx_gs(mgx_ctx *c, int level, int sweeps) {
    if (!c || level < 0 || level >= c->L || sweeps < 0) return fail(MGX_E_ARG, "mgx_gs: bad args");
    if (c->dist) return no_dist(c, "mgx_gs");
    drop_spec(c);
    return op_gs(c, level, sweeps);
}
int mgx_residual_norm(mgx_ctx *c, int level, double *norm) {
    if (!c || level < 0 || level >= c->L || !norm) return fail(MGX_E_ARG, "mgx_residual_norm: bad args");
    if (c->dist) {
        if (level != 0) return no_dist(c, "mgx_residual_norm");
        return dist_residual_norm(c, norm);
    }
    return op_residual_norm(c, level, norm);
}
int mgx_restrict(mgx_ctx *c, int level) {
    if (!c || level < 0 || level >= c->L - 1) return fail(MGX_E_ARG, "mgx_restrict: bad level");
    if (c->dist) return no_dist(c, "mgx_restrict");
    drop_spec(c);
    return op_restrict(c, level);
}
int mgx_prolong_add(mgx_ctx *c, int level) {
    if (!c || level < 0 || level >= c->L - 1) return fail(MGX_E_ARG, "mgx_prolong_add: bad level");
    if (c->dist) return no_dist(c, "mgx_prolong_add");
    drop_spec(c);
    return op_prolong_add(c, level);
}
// A pending next-step state (mgx_step) is only valid for the next mgx_step.
static void drop_step_spec(mgx_ctx *c) {
    if (c->step_spec) drop_spec(c);
}
int mgx_vcycle(mgx_ctx *c) {
    if (!c) return fail(MGX_E_ARG, "null ctx");
    drop_step_spec(c);
    if (c->dist) return dist_vcycle(c, nullptr);
    return op_vcycle(c, 0);
}
int mgx_mg_outer(mgx_ctx *c, double tol, int *cycles, double *res0, double *res) {
    if (!c) return fail(MGX_E_ARG, "null ctx");
    drop_step_spec(c);
    return op_mg_outer(c, tol, cycles, res0, res);
}
// tuning key "step_cross": 1 (default) = mgx_step's last cycle also forms the
// next step's rhs, initial norm and first pre-smoothing (cross pass in step
// mode), consumed by the next mgx_step; 0 = each step starts with its own
// rhs + norm pass
long g_step_cross = 1;

// Step mode needs a second finest-level rhs (the next step's, written by the
// cross pass).  It is allocated on first use, outside any pass; when HBM is
// too short for it (N=65536 on one GPU: the towers take ~265 of 288 GB) the
// context runs the plain schedule instead -- the same results, one pass more
// per step.
static bool step_rhs_alt(mgx_ctx *c) {
    Level &L = c->lv[0];
    if (L.rhs_alt) return true;
    if (c->no_rhs_alt || !cross_ok(c) || !mgx::xstep_supported(L.n)) return false;
    const size_t bytes = sizeof(double) * (size_t)(L.n + 1) * (size_t)L.pitch;
    if (hipMalloc(&L.rhs_alt, bytes) != hipSuccess) {
        (void)hipGetLastError();   // out of memory is not an error here
        L.rhs_alt = nullptr;
        c->no_rhs_alt = true;
        return false;
    }
    // zero boundary: compute_rhs writes the interior only
    if (hipMemsetAsync(L.rhs_alt, 0, bytes, c->stream) != hipSuccess) {
        (void)hipFree(L.rhs_alt);
        L.rhs_alt = nullptr;
        c->no_rhs_alt = true;
        return false;
    }
    return true;
}

static int step_impl(mgx_ctx *c, double tol, int *cycles, bool prepare_next) {
    // compute_rhs and mg_outer's initial norm in one pass (timestepper,
    // multigrid.cpp:168-170), with the first pre-smoothing where it fuses --
    // or already done by the previous step's last cross pass
    double res0 = 0;
    if (c->step_spec && !c->dist) {
        Level &L = c->lv[0];
        std::swap(L.rhs, L.rhs_alt);
        res0 = c->step_res0;
        c->step_spec = false;   // lv[0].spec and lv[1]'s rhs stay: the first cycle's
    } else if (c->dist) {
        CHK(dist_rhs_norm(c, &res0));
    } else if (step_fusable(c)) {
        CHK(op_rhs_norm_pre(c, &res0));
    } else {
        CHK(op_rhs_norm(c, &res0));
    }
    c->step_next = prepare_next && g_step_cross != 0 && !c->dist && step_rhs_alt(c);
    const int rc = op_mg_outer(c, tol, cycles, nullptr, nullptr, &res0);
    c->step_next = false;
    return rc;
}
int mgx_step(mgx_ctx *c, double tol, int *cycles) {
    if (!c) return fail(MGX_E_ARG, "null ctx");
    return step_impl(c, tol, cycles, true);
}
int mgx_run_cycles(mgx_ctx *c, int cycles, double *res) {
    if (!c || cycles < 0) return fail(MGX_E_ARG, "mgx_run_cycles: bad args");
    drop_step_spec(c);
    double r = 0;
    for (int k = 0; k < cycles; ++k) CHK(cycle_norm(c, &r, /*store_post=*/k == cycles - 1));
    if (res) *res = r;
    return MGX_OK;
}

int mgx_level_n(mgx_ctx *c, int level, long *n) {
    if (!c || !n || level < 0 || level >= c->L) return fail(MGX_E_ARG, "mgx_level_n: bad args");
    *n = c->N >> level;
    return MGX_OK;
}
int mgx_coarse_iterations(mgx_ctx *c, long *iters) {
    if (!c || !iters) return fail(MGX_E_ARG, "bad args");
    if (c->dist) c = dist_sub(c, 0);   // every rank runs the same replicated coarse solve
    HIPCHK(hipMemcpyAsync(c->hscal + 2, c->dscal + 2, 2 * sizeof(double), hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    *iters = (long)(c->hscal[2] + c->hscal[4]);
    return MGX_OK;
}
int mgx_stream(mgx_ctx *c, void **stream) {
    if (!c || !stream) return fail(MGX_E_ARG, "bad args");
    *stream = (void *)c->stream;
    return MGX_OK;
}
int mgx_synchronize(mgx_ctx *c) {
    if (!c) return fail(MGX_E_ARG, "null ctx");
    // (partitioned: the side stream's exchanges too -- no RCCL operation of
    // the context is in flight when this returns)
    if (c->dist) CHK(dist_settle(c));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MGX_OK;
}

int mgx_profile_enable(mgx_ctx *c, int on) {
    if (!c) return fail(MGX_E_ARG, "null ctx");
    CHK(prof_flush(c));
    if (on < 0 || on > 2) return fail(MGX_E_ARG, "mgx_profile_enable: on must be 0, 1 or 2");
    c->prof = on;
    // the replicated levels of a partitioned context are never the finest
    for (int i = 0; i < dist_nsub(c); ++i)
        CHK(mgx_profile_enable(dist_sub(c, i), on == 1 ? 1 : 0));
    return MGX_OK;
}
int mgx_profile_reset(mgx_ctx *c) {
    if (!c) return fail(MGX_E_ARG, "null ctx");
    CHK(prof_flush(c));
    memset(c->sum_ms, 0, sizeof(c->sum_ms));
    memset(c->sum_bytes, 0, sizeof(c->sum_bytes));
    memset(c->sum_cbytes, 0, sizeof(c->sum_cbytes));
    memset(c->count, 0, sizeof(c->count));
    for (int i = 0; i < dist_nsub(c); ++i) CHK(mgx_profile_reset(dist_sub(c, i)));
    return MGX_OK;
}
// Partitioned contexts: the replicated levels' launches (sub-contexts, level
// numbers shifted by the first replicated level) are included.
int mgx_profile_get_ex(mgx_ctx *c, int kind, int level, long *launches, double *ms,
                       double *bytes, double *cbytes) {
    if (!c || kind < 0 || kind >= MGX_K_COUNT || level >= 64)
        return fail(MGX_E_ARG, "mgx_profile_get: bad args");
    CHK(prof_flush(c));
    long n = 0;
    double t = 0, b = 0, cb = 0;
    for (int l = 0; l < 64; ++l) {
        if (level >= 0 && l != level) continue;
        n += c->count[kind][l];
        t += c->sum_ms[kind][l];
        b += c->sum_bytes[kind][l];
        cb += c->sum_cbytes[kind][l];
    }
    const int la = dist_la(c);
    for (int i = 0; i < dist_nsub(c); ++i) {
        if (level >= 0 && level < la) break;
        long sn = 0;
        double st = 0, sb = 0, scb = 0;
        CHK(mgx_profile_get_ex(dist_sub(c, i), kind, level < 0 ? -1 : level - la, &sn, &st, &sb,
                               &scb));
        n += sn;
        t += st;
        b += sb;
        cb += scb;
    }
    if (launches) *launches = n;
    if (ms) *ms = t;
    if (bytes) *bytes = b;
    if (cbytes) *cbytes = cb;
    return MGX_OK;
}
int mgx_profile_get(mgx_ctx *c, int kind, int level, long *launches, double *ms, double *bytes) {
    return mgx_profile_get_ex(c, kind, level, launches, ms, bytes, nullptr);
}

// ---- timestepper (multigrid.cpp:124-186)
int mgx_timestepper_ex(double *uT, const double *u0, const double *v1, const double *v2,
                       double nu, int maxlvl, long n, double dt, double T, double dx, double tol,
                       const mgx_options *opt, int *cycles_per_step) {
    (void)dx;   // the context derives dx = 1/n (multigrid.cpp:194)
    if (!uT || !u0 || !v1 || !v2) return fail(MGX_E_ARG, "mgx_timestepper: null array");
    mgx_ctx *c = nullptr;
    CHK(mgx_create(&c, n, maxlvl, dt, nu, opt));
    int rc = mgx_upload(c, u0, v1, v2);
    const int steps = (int)(T / dt);   // multigrid.cpp:165
    for (int it = 0; rc == MGX_OK && it < steps; ++it) {
        int cyc = 0;
        rc = step_impl(c, tol, &cyc, /*prepare_next=*/it + 1 < steps);
        if (rc == MGX_E_NOCONV) {
            // multigrid.cpp:117-119 only warns; keep stepping
            printf("multigrid did not converge in %d cycles\n", c->opt.max_cycle);
            rc = MGX_OK;
        }
        if (cycles_per_step) cycles_per_step[it] = cyc;
    }
    if (rc == MGX_OK) rc = mgx_download(c, uT);
    std::string keep = g_err;
    mgx_destroy(c);
    g_err = keep;
    return rc;
}

int mgx_timestepper(double *uT, const double *u0, const double *v1, const double *v2, double nu,
                    int maxlvl, long n, double dt, double T, double dx, double tol, int shape) {
    mgx_options o;
    mgx_default_options(&o);
    o.shape = shape;
    return mgx_timestepper_ex(uT, u0, v1, v2, nu, maxlvl, n, dt, T, dx, tol, &o, nullptr);
}

}  // extern "C"

// ---- reference problem setup (multigrid.cpp:206-233), host, glibc libm
#include <thread>
// Rows [r0, r1) of the reference problem (multigrid.cpp:206-233) into arrays
// holding just those rows; bitwise the rows of the full initialisation.
static int init_rows(double *u0, double *v1, double *v2, long N, long r0, long r1,
                     int nthreads) {
    const double PI = 3.1415926535897932;   // multigrid.cpp:14
    const double dx = 1.0 / N;
    const double x0 = 0.2, y0 = 0.4, sigma = 100.0, kx = 1.0 * PI, ky = 1.0 * PI;
    const long w = N + 1;
    int nt = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
    if (nt < 1) nt = 1;
    if (nt > r1 - r0) nt = (int)std::max<long>(1, r1 - r0);
    auto rows = [&](long a, long b) {
        for (long i = a; i < b; ++i) {
            const double xi = (double)i;
            const long o = (i - r0) * w;
            for (long j = 0; j < w; ++j) {
                const double yj = (double)j;
                u0[o + j] = std::exp(-sigma * ((xi * dx - x0) * (xi * dx - x0) +
                                               (yj * dx - y0) * (yj * dx - y0)));
                v1[o + j] = -ky * std::sin(kx * xi * dx) * std::cos(ky * yj * dx);
                v2[o + j] = kx * std::cos(kx * xi * dx) * std::sin(ky * yj * dx);
            }
        }
    };
    std::vector<std::thread> th;
    const long per = (r1 - r0 + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        long a = r0 + t * per, b = std::min(r1, a + per);
        if (a < b) th.emplace_back(rows, a, b);
    }
    for (auto &x : th) x.join();
    // zero boundary, multigrid.cpp:227-233 (row N, column 0 stays: the
    // reference's loops skip that corner)
    auto in = [&](long i) { return i >= r0 && i < r1; };
    for (long i = 0; i < N; ++i) {
        if (in(0)) u0[(0 - r0) * w + i] = 0.0;
        if (in(i)) u0[(i - r0) * w + N] = 0.0;
        if (in(N)) u0[(N - r0) * w + i + 1] = 0.0;
        if (in(i)) u0[(i - r0) * w] = 0.0;
    }
    return MGX_OK;
}

extern "C" int mgx_init_problem(double *u0, double *v1, double *v2, long N, int nthreads) {
    if (!u0 || !v1 || !v2 || N < 1) return fail(MGX_E_ARG, "mgx_init_problem: bad args");
    return init_rows(u0, v1, v2, N, 0, N + 1, nthreads);
}

extern "C" int mgx_init_problem_rows(double *u0, double *v1, double *v2, long N, long r0,
                                     long r1, int nthreads) {
    if (!u0 || !v1 || !v2 || N < 1 || r0 < 0 || r1 > N + 1 || r0 >= r1)
        return fail(MGX_E_ARG, "mgx_init_problem_rows: bad args");
    return init_rows(u0, v1, v2, N, r0, r1, nthreads);
}

// The reference's uT text writer (multigrid.cpp:269-284: fprintf "%d\t%d\t%f\n",
// i outer, j inner) for rows [r0, r1) held in `rows` ((r1-r0) x (N+1)), so a
// row-partitioned run writes its output block by block: rank r appends its
// owned rows in rank order and the file is byte-identical to the whole-grid
// writer.  Lines are formatted by nthreads threads, written in order.
extern "C" int mgx_write_uT(const char *path, const double *rows, long N, long r0, long r1,
                            int append, int nthreads) {
    if (!path || !rows || N < 1 || r0 < 0 || r1 > N + 1 || r0 > r1)
        return fail(MGX_E_ARG, "mgx_write_uT: bad args");
    FILE *f = fopen(path, append ? "ab" : "wb");
    if (!f) return fail(MGX_E_ARG, std::string("mgx_write_uT: cannot open ") + path);
    int nt = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
    nt = std::max(1, std::min(nt, 64));
    const long w = N + 1, per = 8;   // rows per thread per batch
    std::vector<std::string> buf(nt);
    int rc = MGX_OK;
    for (long b0 = r0; b0 < r1 && rc == MGX_OK; b0 += per * nt) {
        auto fmt = [&](int t) {
            std::string &s = buf[t];
            s.clear();
            char line[400];   // "%f" of DBL_MAX is 316 characters
            const long a = b0 + t * per, e = std::min(r1, a + per);
            for (long i = a; i < e; ++i)
                for (long j = 0; j < w; ++j) {
                    const int k = snprintf(line, sizeof line, "%d\t%d\t%f\n", (int)i, (int)j,
                                           rows[(i - r0) * w + j]);
                    s.append(line, k);
                }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(fmt, t);
        fmt(0);
        for (auto &x : th) x.join();
        for (int t = 0; t < nt && rc == MGX_OK; ++t)
            if (!buf[t].empty() && fwrite(buf[t].data(), 1, buf[t].size(), f) != buf[t].size())
                rc = fail(MGX_E_ARG, std::string("mgx_write_uT: write failed: ") + path);
    }
    if (fclose(f) != 0 && rc == MGX_OK) rc = fail(MGX_E_ARG, "mgx_write_uT: close failed");
    return rc;
}

// sepvel.h's exact rank-1 factorisation, for tests: v (rows x (n+1)) ==
// fl(a[i] * b[j]) bitwise -> 1 (a, b filled), else 0.  Host only.
extern "C" int mgx_factor_velocity(const double *v, long rows, long n, double smin, double *a,
                                   double *b) {
    if (!v || !a || !b || rows < 1 || n < 1) return fail(MGX_E_ARG, "mgx_factor_velocity: bad args");
    return mgxsep::factor_rank1(v, rows, n + 1, n + 1, smin, a, b) ? 1 : 0;
}

// whether the context's finest level holds velocity factors (its cross pass
// reads rhs and u only)
extern "C" int mgx_velocity_factored(mgx_ctx *c, int *factored) {
    if (!c || !factored) return fail(MGX_E_ARG, "mgx_velocity_factored: bad args");
    if (c->dist) {
        *factored = dist_velocity_mask(c);
        return MGX_OK;
    }
    int f = (!c->lv.empty() && c->lv[0].sa1) ? 1 : 0;
    for (size_t l = 1; l < c->lv.size() && l < 31; ++l)
        if (c->lv[l].vgen && mgxi::g_vgen) f |= 1 << l;
    *factored = f;
    return MGX_OK;
}

// ---- tuning knobs (process-wide)
extern "C" int mgx_set_tuning(const char *key, long value) {
    if (!key) return fail(MGX_E_ARG, "mgx_set_tuning: null key");
    ++mgxi::g_tuning_epoch;   // captured sub-cycles of the old settings are stale
    if (!strcmp(key, "graph_level")) {
        if (value < 0) return fail(MGX_E_ARG, "graph_level must be >= 0");
        mgxi::g_graph_level = value;
        return MGX_OK;
    }
    if (!strcmp(key, "tile_max_n")) {
        mgx::set_tile_max_n(value);
        return MGX_OK;
    }
    if (!strcmp(key, "cross_cycle")) {
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "cross_cycle must be 0 or 1");
        mgxi::g_cross_cycle = value;
        return MGX_OK;
    }
    if (!strcmp(key, "dist_overlap")) {
        if (value < -1 || value > 2) return fail(MGX_E_ARG, "dist_overlap must be -1, 0, 1 or 2");
        mgxi::g_dist_overlap = value;
        return MGX_OK;
    }
    if (!strcmp(key, "dist_local_side")) {
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "dist_local_side must be 0 or 1");
        mgxi::g_dist_local_side = value;
        return MGX_OK;
    }
    if (!strcmp(key, "coarse_fuse")) {
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "coarse_fuse must be 0 or 1");
        mgxi::g_coarse_fuse = value;
        return MGX_OK;
    }
    if (!strcmp(key, "wpair")) {
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "wpair must be 0 or 1");
        mgxi::g_wpair = value;
        return MGX_OK;
    }
    if (!strcmp(key, "dist_comm_chain")) {   // test hook (dist.hip)
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "dist_comm_chain must be 0 or 1");
        mgxi::g_dist_comm_chain = value;
        return MGX_OK;
    }
    if (!strcmp(key, "dist_min_rows")) {
        if (value < 16 || (value & 1)) return fail(MGX_E_ARG, "dist_min_rows must be even, >= 16");
        mgxi::g_dist_min_rows = value;
        return MGX_OK;
    }
    if (!strcmp(key, "xfast")) {
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "xfast must be 0 or 1");
        mgx::set_xfast(value);
        return MGX_OK;
    }
    if (!strcmp(key, "tile32_min_n")) {
        if (value < 0) return fail(MGX_E_ARG, "tile32_min_n must be >= 0");
        mgx::set_tile32_min_n(value);
        return MGX_OK;
    }
    if (!strcmp(key, "tile_xcd")) {
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "tile_xcd must be 0 or 1");
        mgx::set_tile_xcd(value);
        return MGX_OK;
    }
    if (!strcmp(key, "march_order")) {
        if (value < 0 || value > 3) return fail(MGX_E_ARG, "march_order must be 0..3");
        mgx::set_march_order(value);
        return MGX_OK;
    }
    if (!strcmp(key, "march_min_rows")) {
        if (value < 8) return fail(MGX_E_ARG, "march_min_rows must be >= 8");
        mgx::set_march_min_rows(value);
        return MGX_OK;
    }
    if (!strcmp(key, "xtile_max_rows")) {
        if (value < 0) return fail(MGX_E_ARG, "xtile_max_rows must be >= 0");
        mgx::set_xtile_max_rows(value);
        return MGX_OK;
    }
    if (!strcmp(key, "step_cross")) {
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "step_cross must be 0 or 1");
        g_step_cross = value;
        return MGX_OK;
    }
    if (!strcmp(key, "post_only")) {
        if (value < -1) return fail(MGX_E_ARG, "post_only must be >= -1");
        mgxi::g_post_only = value;
        return MGX_OK;
    }
    if (!strcmp(key, "post_predict")) {
        if (value < -1) return fail(MGX_E_ARG, "post_predict must be >= -1");
        mgxi::g_post_predict = (double)value;
        return MGX_OK;
    }
    if (!strcmp(key, "march_seg")) {
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "march_seg must be 0 or 1");
        mgx::set_march_seg(value);
        return MGX_OK;
    }
    if (!strcmp(key, "step_fuse")) {
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "step_fuse must be 0 or 1");
        mgxi::g_step_fuse = value;
        return MGX_OK;
    }
    if (!strcmp(key, "coarse_lds")) {
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "coarse_lds must be 0 or 1");
        mgx::set_coarse_lds(value);
        return MGX_OK;
    }
    if (!strcmp(key, "sep_velocity")) {
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "sep_velocity must be 0 or 1");
        mgxi::g_sep_velocity = value;
        return MGX_OK;
    }
    if (!strcmp(key, "vgen")) {
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "vgen must be 0 or 1");
        mgxi::g_vgen = value;
        return MGX_OK;
    }
    if (!strcmp(key, "zero_rows")) {
        if (value != 0 && value != 1) return fail(MGX_E_ARG, "zero_rows must be 0 or 1");
        mgxi::g_zero_rows = value;
        return MGX_OK;
    }
    if (!strcmp(key, "march_tile_rows")) {
        if (value < 0) return fail(MGX_E_ARG, "march_tile_rows must be >= 0");
        mgx::set_march_tile_rows(value);
        return MGX_OK;
    }
    return fail(MGX_E_ARG, std::string("mgx_set_tuning: unknown key ") + key);
}
extern "C" int mgx_get_tuning(const char *key, long *value) {
    if (!key || !value) return fail(MGX_E_ARG, "mgx_get_tuning: null argument");
    if (!strcmp(key, "graph_level")) {
        *value = mgxi::g_graph_level;
        return MGX_OK;
    }
    if (!strcmp(key, "graph_captures") || !strcmp(key, "graph_replays")) {
        *value = key[6] == 'c' ? mgxi::g_graph_captures : mgxi::g_graph_replays;
        return MGX_OK;
    }
    if (!strcmp(key, "tile_max_n")) {
        *value = mgx::get_tile_max_n();
        return MGX_OK;
    }
    if (!strcmp(key, "cross_cycle")) {
        mgxi::cross_cycle_on();
        *value = mgxi::g_cross_cycle;
        return MGX_OK;
    }
    if (!strcmp(key, "dist_overlap")) {
        *value = mgxi::g_dist_overlap;
        return MGX_OK;
    }
    if (!strcmp(key, "dist_local_side")) {
        *value = mgxi::g_dist_local_side;
        return MGX_OK;
    }
    if (!strcmp(key, "dist_comm_chain")) {
        *value = mgxi::g_dist_comm_chain;
        return MGX_OK;
    }
    if (!strcmp(key, "coarse_fuse")) {
        *value = mgxi::g_coarse_fuse;
        return MGX_OK;
    }
    if (!strcmp(key, "wpair")) {
        *value = mgxi::g_wpair;
        return MGX_OK;
    }
    if (!strcmp(key, "dist_min_rows")) {
        *value = mgxi::g_dist_min_rows;
        return MGX_OK;
    }
    if (!strcmp(key, "xfast")) {
        *value = mgx::get_xfast();
        return MGX_OK;
    }
    if (!strcmp(key, "tile32_min_n")) {
        *value = mgx::get_tile32_min_n();
        return MGX_OK;
    }
    if (!strcmp(key, "tile_xcd")) {
        *value = mgx::get_tile_xcd();
        return MGX_OK;
    }
    if (!strcmp(key, "march_order")) {
        *value = mgx::get_march_order();
        return MGX_OK;
    }
    if (!strcmp(key, "march_min_rows")) {
        *value = mgx::get_march_min_rows();
        return MGX_OK;
    }
    if (!strcmp(key, "xtile_max_rows")) {
        *value = mgx::get_xtile_max_rows();
        return MGX_OK;
    }
    if (!strcmp(key, "step_cross")) {
        *value = g_step_cross;
        return MGX_OK;
    }
    if (!strcmp(key, "post_only")) {
        *value = mgxi::g_post_only;
        return MGX_OK;
    }
    if (!strcmp(key, "post_predict")) {
        *value = (long)mgxi::g_post_predict;
        return MGX_OK;
    }
    if (!strcmp(key, "march_seg")) {
        *value = mgx::get_march_seg();
        return MGX_OK;
    }
    if (!strcmp(key, "step_fuse")) {
        *value = mgxi::g_step_fuse;
        return MGX_OK;
    }
    if (!strcmp(key, "coarse_lds")) {
        *value = mgx::get_coarse_lds();
        return MGX_OK;
    }
    if (!strcmp(key, "sep_velocity")) {
        *value = mgxi::g_sep_velocity;
        return MGX_OK;
    }
    if (!strcmp(key, "vgen")) {
        *value = mgxi::g_vgen;
        return MGX_OK;
    }
    if (!strcmp(key, "zero_rows")) {
        *value = mgxi::g_zero_rows;
        return MGX_OK;
    }
    if (!strcmp(key, "march_tile_rows")) {
        *value = mgx::get_march_tile_rows();
        return MGX_OK;
    }
    return fail(MGX_E_ARG, std::string("mgx_get_tuning: unknown key ") + key);
}

// Streaming-bandwidth probe (a measured ceiling beside the spec).
extern "C" int mgx_stream_bandwidth(long bytes_per_stream, int nin, int reps, double *GBs) {
    if (bytes_per_stream < (1 << 20) || (nin != 1 && nin != 4) || reps < 1 || !GBs)
        return fail(MGX_E_ARG, "mgx_stream_bandwidth: bad args");
    const long n2 = bytes_per_stream / 16;
    const size_t bytes = (size_t)n2 * 16;
    double *buf[5] = {};
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = MGX_OK;
    int dev = 0, cus = 0;
    auto cleanup = [&]() {
        for (double *b : buf) (void)hipFree(b);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        if (s) (void)hipStreamDestroy(s);
    };
    for (int k = 0; k <= nin; ++k)
        if (hipMalloc(&buf[k], bytes) != hipSuccess ||
            hipMemset(buf[k], 0, bytes) != hipSuccess) {
            cleanup();
            return fail(MGX_E_HIP, "mgx_stream_bandwidth: alloc");
        }
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipStreamCreate(&s) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess) {
        cleanup();
        return fail(MGX_E_HIP, "mgx_stream_bandwidth: stream/events");
    }
    // one 16-B element per lane (kernels.hip k_stream)
    const int grid = (int)std::min<long>((n2 + 255) / 256, 1L << 30);
    double *a = buf[0], *b = buf[nin > 1 ? 1 : 0], *c = buf[nin > 1 ? 2 : 0],
           *d = buf[nin > 1 ? 3 : 0], *o = buf[nin];
    mgx::launch_stream(a, b, c, d, o, n2, nin, grid, s);   // warm-up
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < reps; ++r) mgx::launch_stream(a, b, c, d, o, n2, nin, grid, s);
    (void)hipEventRecord(e1, s);
    float ms = 0.f;
    if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess)
        rc = fail(MGX_E_HIP, "mgx_stream_bandwidth: timing");
    else
        *GBs = (double)bytes * (nin + 1) * reps / (ms * 1e-3) / 1e9;
    cleanup();
    return rc;
}
