// ctx.h -- internal: the solver context shared by mgx.hip (single GPU) and
// dist.hip (row-partitioned, multi-GPU).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/mgx.h"
#include "kernels.h"

namespace mgxi {

int fail(int code, const std::string &msg);
int check_launch(const char *what);

#define HIPCHK(expr)                                                                     \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return ::mgxi::fail(MGX_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define CHK(expr)              \
    do {                       \
        int rc_ = (expr);      \
        if (rc_) return rc_;   \
    } while (0)

struct Level {
    long n = 0, pitch = 0;
    double *u[3] = {nullptr, nullptr, nullptr};   // u[2]: finest level, cross-cycle pass
    int cur = 0;
    bool zero = false;   // u is logically all zeros (multigrid.cpp:77), not yet written
    // finest level only: index of the buffer holding the NEXT cycle's
    // pre-smoothed u (written by the cross-cycle pass, with rhs[1] restricted
    // from it and u[1] flagged zero), or -1
    int spec = -1;
    int xin = -1;   // finest level: the input buffer of the last cross-cycle pass
    int nxt() const { return cur == 0 ? 1 : 0; }   // ping-pong partner of cur
    double *rhs = nullptr, *v1 = nullptr, *v2 = nullptr;
    // finest level: the next time step's rhs (step mode); coarsest level (n <=
    // 64, L >= 3): the rhs a W-cycle's fused pair pass restricts into while its
    // workgroups still read the current one for the fused coarsest solve
    double *rhs_alt = nullptr;
    // exact rank-1 factors of v1 / v2 (sepvel.h; row factors n+1, column
    // factors pitch, zero padded), or null: the passes that take them read
    // the 2-D v1 / v2 from HBM only where no factors exist
    double *sa1 = nullptr, *sb1 = nullptr, *sa2 = nullptr, *sb2 = nullptr;
    // rows >= vz of v1 and v2 are all zeros (found at upload): the row march
    // reads them from mgx_ctx::zrow (L2-resident) instead of HBM
    int vz = 0x7fffffff;
    // levels 1-2 of the reference tower, levels >= 1 of the correct one: v1 /
    // v2 equal the generator's entries from the finest factors (checked at
    // upload, stencil.h vg_col)
    bool vgen = false;
    mgx::Coef coef{};
    double M() const { return double(n + 1) * double(n + 1); }
    // compulsory bytes of v1 + v2 of this level (the zero rows cost no HBM)
    double Mv() const { return double(std::min<long>(n + 1, vz)) * double(n + 1); }
    double *U() const { return u[cur]; }
};

struct ProfRec {
    int kind, level;
    double bytes;    // canonical algorithmic bytes (SURVEY 8d per-op model)
    double cbytes;   // compulsory bytes: every array the launch reads or writes, once
    hipEvent_t e0, e1;
};

struct Dist;   // dist.hip

}  // namespace mgxi

struct mgx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = true;
    long N = 0;
    int L = 0;
    double dt = 0, nu = 0;
    mgx_options opt{};
    std::vector<mgxi::Level> lv;
    double *partials = nullptr;   // norm partial sums
    double *dscal = nullptr;      // [0] norm, [2..3] coarse stats (iterations, last norm)
    double *hscal = nullptr;      // pinned host mirror
    double *stage[2] = {nullptr, nullptr};   // reference-layout (N+1)^2 staging
    double *zrow = nullptr;   // one row of zeros (finest pitch): Level::vz rows read it
    double2 *vga = nullptr;   // VGen::a of the Level::vgen levels, N+2 pairs
    mgxi::Dist *dist = nullptr;   // row-partitioned multi-GPU state (dist.hip)
    // mg_outer's cycle predicted to be the last: its finest level runs the
    // post-smoothing alone, not the cross pass (no next-cycle pre-smoothing)
    bool post_only = false;
    // the coarsest solve of level cf_level (cf_reps solves) deferred into the
    // prolongation tile pass of the level above (tuning key "coarse_fuse");
    // -1: none pending
    int cf_level = -1, cf_reps = 0;
    // time-step mode: inside mgx_step (step_next) the last cycle's cross pass
    // also forms the next step's rhs (lv[0].rhs_alt), initial norm
    // (step_res0) and first pre-smoothing + restriction (lv[0].spec, lv[1]
    // rhs); step_spec = that state is ready for the next mgx_step
    bool step_next = false, step_spec = false;
    bool no_rhs_alt = false;   // the step-mode rhs did not fit in HBM: plain schedule
    // tuning key "graph_level": the sub-cycle below a level replayed as a
    // captured hipGraph, one per entry state (mgx.hip graph_vcycle)
    struct Graph {
        std::vector<long> key, end;
        hipGraphExec_t exec = nullptr;
    };
    std::vector<Graph> graphs;
    bool capturing = false;
    double step_res0 = 0;
    // profiling
    int prof = 0;   // 0 off, 1 every launch, 2 finest-level launches only
    std::vector<mgxi::ProfRec> pending;
    std::vector<hipEvent_t> pool;
    double sum_ms[MGX_K_COUNT][64] = {};
    double sum_bytes[MGX_K_COUNT][64] = {};
    double sum_cbytes[MGX_K_COUNT][64] = {};
    long count[MGX_K_COUNT][64] = {};
};

namespace mgxi {

hipEvent_t take_event(mgx_ctx *c);

// A launch whose lambda declined (launched nothing: the caller saw a negative
// block count) drops the record it pushed, so profiles count real launches.
inline void unlaunch(mgx_ctx *c, size_t pending_before) {
    while (c->pending.size() > pending_before) {
        c->pool.push_back(c->pending.back().e0);
        c->pool.push_back(c->pending.back().e1);
        c->pending.pop_back();
    }
}
// Launch helper: records HIP events around the launch when profiling is on.
// bytes: canonical algorithmic bytes of the reference ops the launch does
// (SURVEY 8d); cbytes: its compulsory bytes (each array it must read or write,
// once) -- the roofline denominator of a fused pass.
template <class F>
int launch(mgx_ctx *c, int kind, int level, double bytes, double cbytes, F &&f) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool rec = c->prof == 1 || (c->prof == 2 && level == 0);
    if (rec) {
        e0 = take_event(c);
        e1 = take_event(c);
        if (e0) (void)hipEventRecord(e0, c->stream);
    }
    f();
    CHK(check_launch("kernel launch"));
    if (rec && e0 && e1) {
        (void)hipEventRecord(e1, c->stream);
        c->pending.push_back({kind, level, bytes, cbytes, e0, e1});
    }
    return MGX_OK;
}
// single-op launches: canonical == compulsory
template <class F>
int launch(mgx_ctx *c, int kind, int level, double bytes, F &&f) {
    return launch(c, kind, level, bytes, bytes, static_cast<F &&>(f));
}

int prof_flush(mgx_ctx *c);
int materialize(mgx_ctx *c, int l);
int read_norm(mgx_ctx *c, double *norm);
// store_post: see op_cross (false only between cycles of one run_cycles call)
int op_vcycle(mgx_ctx *c, int l, double *norm = nullptr, bool store_post = true);
int op_rhs(mgx_ctx *c);
int op_residual_norm(mgx_ctx *c, int l, double *norm, double bytes_per_pt = 48.0);
int build_tower(mgx_ctx *c);
// Level::vz of levels 1..L-1 from the built tower (the first row from which
// every row of v1 and v2 is zero)
int find_zero_rows(mgx_ctx *c);
// velocity factors of level 0 from host copies of v1 / v2 (rows [r0, r0+rows)
// of width n+1); false: not separable (or "sep_velocity" off), nothing set
bool factor_velocity(const double *v1, const double *v2, long n, long r0, long rows, double smin,
                     std::vector<double> &a1, std::vector<double> &b1, std::vector<double> &a2,
                     std::vector<double> &b2, long *js1 = nullptr, long *js2 = nullptr);
int set_level_factors(Level &L, long row0, const std::vector<double> &a1,
                      const std::vector<double> &b1, const std::vector<double> &a2,
                      const std::vector<double> &b2, hipStream_t s);
void free_level_factors(Level &L);
extern long g_sep_velocity;
extern long g_vgen;   // tuning key "vgen" (mgx.hip)
void free_ctx(mgx_ctx *c);
// Create a single-GPU context; stream != nullptr: borrow that stream.
int create_ctx(mgx_ctx **out, long n, int maxlvl, double dt, double nu, const mgx_options *opt,
               hipStream_t stream);
int upload_ctx(mgx_ctx *c, const double *u0, const double *v1, const double *v2,
               hipMemcpyKind kind);

// dist.hip entry points used by the C ABI
int dist_upload(mgx_ctx *c, const double *u0, const double *v1, const double *v2,
                hipMemcpyKind kind);
int dist_download(mgx_ctx *c, double *u, hipMemcpyKind kind);
int dist_owned_rows(mgx_ctx *c, int part, int *ra, int *rb);
int dist_download_rows(mgx_ctx *c, int part, double *out, hipMemcpyKind kind);
int dist_rhs(mgx_ctx *c);
int dist_rhs_norm(mgx_ctx *c, double *res0);
int dist_vcycle(mgx_ctx *c, double *norm, bool store_post = true);
// partitioned level 0 runs the cross-cycle pass; recompute its unstored u_post
bool dist_post_predictable(mgx_ctx *c);
int dist_redo_post(mgx_ctx *c);
int dist_residual_norm(mgx_ctx *c, double *norm);
void dist_free(mgx_ctx *c);
// replicated coarse-level contexts of a partitioned context (one per local part)
int dist_nsub(mgx_ctx *c);
mgx_ctx *dist_sub(mgx_ctx *c, int i);
int dist_la(mgx_ctx *c);
int dist_velocity_mask(mgx_ctx *c);   // mgx_velocity_factored of a partitioned context
int dist_settle(mgx_ctx *c);   // join the side stream's exchanges into the compute stream
// levels whose row blocks would be shorter than this are replicated (tuning
// key "dist_min_rows", default 256)
extern long g_dist_min_rows;
// tuning key "dist_overlap" (dist.hip): finest-level ghost exchange on a second
// stream beside the interior of the cross-cycle pass
extern long g_dist_overlap;
// tuning key "dist_local_side" (dist.hip): virtual ranks' early exchanges on
// the compute stream (0) or the second stream (1)
extern long g_dist_local_side;
extern long g_dist_comm_chain;   // tuning key "dist_comm_chain" (test hook)
// tuning key "cross_cycle" (mgx.hip); levels with n >= kCrossMinN can use it
bool cross_cycle_on();
constexpr long kCrossMinN = 4096;

}  // namespace mgxi
