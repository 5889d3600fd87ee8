// dist.hip -- row-partitioned multi-GPU V-cycle.
//
// Levels 0..la-1 are split into contiguous row blocks, one per rank (even
// block boundaries, so restriction rows 2I and prolongation parents stay
// local).  Each block carries kGhost rows of its neighbours on each side;
// because a fused smoothing pass of E stages is exact on the owned rows
// given E ghost rows (the temporal-blocking cone, kernels.hip k_smooth), ONE
// halo exchange per fused pass is enough -- where a sweep-by-sweep smoother
// needs two per sweep.  Levels la..L-1 (where a block would be small) are
// replicated: the restricted rhs is all-gathered into a full single-GPU
// context on every rank, which runs the rest of the V-cycle redundantly and
// bitwise identically, and the post-smoothing pass of level la-1 prolongs
// from its (full) solution with no further exchange.  The residual norm of
// the finest level is a per-rank partial sum + all-reduce.
//
// Two transports with the same partition logic:
//   * RCCL (mgx_create_dist): one process per GPU, ncclSend/ncclRecv of whole
//     ghost-row blocks (contiguous in the pitched layout) to rank +-1 over
//     xGMI, ncclAllGather / ncclAllReduce -- ONE communicator, and at most one
//     of its operations in flight per rank: each is chained after the
//     previous one (comm_op), whichever of the two streams issues it;
//   * local (mgx_create_local_dist): `world` virtual ranks in one process on
//     one device, exchanges as device-to-device copies -- for testing the
//     partitioned solver against the single-GPU one on a one-GPU machine.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <initializer_list>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ctx.h"
#include "plan.h"

namespace mgxi {

long g_dist_min_rows = 256;
// tuning key "dist_overlap": 1 = every partitioned level's u ghost rows are
// exchanged from a second stream as soon as the pass that wrote them ends --
// the pre-smoothing pass, or the finest level's cross pass -- hidden behind
// the coarser levels of the V-cycle (the level's post pass waits for it, and
// then exchanges only the coarser level's u for its prolongation); 2 = that,
// and the cross pass's remaining u ghost exchange (dist_cross: level 0's when
// it was not exchanged early, level 1's without the communication-avoiding
// post passes) on the second stream too, beside the pass's interior march
// (the bands next to the ghosts go to its edge launch); 0 = every exchange on
// the compute stream; -1
// (default) = 1 on an RCCL communicator, 0 on virtual ranks.  The second
// stream has NO communicator of its own: its exchanges go through the rank's
// one communicator, chained after the previous operation by comm_op (Dist::
// comm), so the overlap is with compute only, never between two RCCL
// operations.  On virtual ranks (one GPU) the early exchange's copies compete
// with the level passes for the same chip and cost 2-3 %; over xGMI it takes
// the level-0 exchange (2 x 16 rows, ~4 MB per rank) off the critical path
// for nothing of the local HBM -- bench.py prices 0 / 1 / 2 (with
// dist_min_rows 128 / 256) on the N-GPU run itself and keeps the fastest for
// its timed region
long g_dist_overlap = -1;
// tuning key "dist_local_side": virtual ranks (one device) run the
// dist_overlap exchanges at their early points ON the compute stream (0,
// default: one chip has no second link to overlap with -- on a second stream
// the copy kernels waited for CUs held by the level passes and each join
// cost a bubble, +5 % per cycle at G = 8) or on the second stream as over
// RCCL (1: exercises the fork / join logic on one GPU).  Bitwise the same.
long g_dist_local_side = 0;
// tuning key "dist_comm_chain": 1 (default) = every RCCL operation of a rank is
// ordered after its previous one (comm_op); 0 = a TEST HOOK that drops the
// chain, so tests/test_gpu_fake_rccl.py can show that the fake RCCL's
// happens-before check catches two operations in flight at once.  Never 0 on
// real peers: NCCL operations of one communicator must not run concurrently.
long g_dist_comm_chain = 1;

// the partition / exchange plan (plan.h, host-only)
using mgxplan::alloc_rows;
using mgxplan::gather_rows;
using mgxplan::ghost_plan;
using mgxplan::kGhost;
using mgxplan::kGhostFine;
using mgxplan::kPostExt;
using mgxplan::plan_rows;
using mgxplan::Xfer;
static int plan_la(long n0, int L, int world) {
    return mgxplan::plan_la(n0, L, world, g_dist_min_rows);
}
static int plan_check(long n0, int l, int world) {
    const std::string e = mgxplan::plan_check(n0, l, world);
    return e.empty() ? MGX_OK : fail(MGX_E_INTERNAL, e);
}

#define NCCLCHK(expr)                                                                    \
    do {                                                                                 \
        ncclResult_t r_ = (expr);                                                        \
        if (r_ != ncclSuccess)                                                           \
            return fail(MGX_E_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

struct PLevel {
    long n = 0, pitch = 0;
    int ra = 0, rb = 0;   // owned rows [ra, rb)
    int lo = 0, hi = 0;   // allocated rows [lo, hi] (owned + ghosts, clipped to [0, n])
    double *u[3] = {nullptr, nullptr, nullptr};   // u[2]: level 0, cross-cycle pass
    int cur = 0;
    int spec = -1;   // level 0: buffer of the next cycle's pre-smoothed u (Level::spec)
    int xin = -1;    // level 0: input buffer of the last cross-cycle pass (Level::xin)
    bool zero = false;
    double *rhs = nullptr, *v1 = nullptr, *v2 = nullptr;
    // level 0: exact velocity factors (sepvel.h) indexed by GLOBAL row / column
    // (full-length arrays, this block's rows filled), or null
    double *sa1 = nullptr, *sb1 = nullptr, *sa2 = nullptr, *sb2 = nullptr;
    int vz = 0x7fffffff;   // Level::vz (global rows)
    bool vgen = false;     // Level::vgen (generated velocity)
    // level 0 of a row-block upload: the columns whose entries are the row
    // factors of v1 / v2 (sepvel.h j*), or -1
    long js1 = -1, js2 = -1;
    mgx::Coef coef{};
    int nxt() const { return cur == 0 ? 1 : 0; }
    // field pointer offset so that F(a) + r*pitch is global row r
    double *F(double *a) const { return a - (long)lo * pitch; }
    double *U() const { return F(u[cur]); }
    size_t bytes() const { return sizeof(double) * (size_t)(hi - lo + 1) * pitch; }
    double Mown() const { return double(rb - ra) * double(n + 1); }
};

struct Part {
    int rank = 0;
    std::vector<PLevel> lv;   // levels 0..la-1
    mgx_ctx *sub = nullptr;   // levels la..L-1, full, replicated
    double *dsum = nullptr;   // device scalar: this rank's partial sum of squares
    double *partials = nullptr;   // this part's norm partials (a split pass keeps them
                                  // between its two launches while other parts run)
    double2 *vga = nullptr;       // mgx_ctx::vga (levels with PLevel::vgen), or null
    hipEvent_t xe0 = nullptr;     // profiling: the start of a split pass
};

struct Dist {
    int world = 1;
    bool local = false;
    int la = 0;
    std::vector<Part> parts;   // local: `world` parts; RCCL: this rank's part
    // ONE communicator for every operation, compute stream and side stream
    // alike.  NCCL runs the operations of a communicator in the order they are
    // issued and they must not overlap; two communicators in flight at once
    // "might work provided they fit within the GPU" and can deadlock otherwise
    // (round-4 verdict).  So every operation goes through comm_op, which chains
    // it after the rank's previous one: ev_comm is recorded after each, and an
    // operation issued on the other stream than its predecessor waits for it.
    ncclComm_t comm = nullptr;
    hipEvent_t ev_comm = nullptr;      // end of this rank's last RCCL operation
    hipStream_t comm_last = nullptr;   // the stream that issued it
    double *hsum = nullptr;    // pinned
    double *dsum_all = nullptr;   // virtual ranks: the parts' sums added (device)
    // dist_overlap: ghost exchanges on a second stream beside the interior pass
    hipStream_t xs = nullptr;
    hipEvent_t ev_fork = nullptr;
    hipEvent_t ev_join = nullptr;   // the side stream's last recorded work
    bool early_pending = false;     // side-stream work the compute stream has not joined
    // dist_overlap, per partitioned level l: the u buffer whose ghost rows the
    // side stream has exchanged (or is exchanging) since it was last written,
    // or -1; ev_lvl[l] marks the end of that exchange, lvl_pending[l] = not yet
    // waited for by the compute stream
    std::vector<int> early_buf;
    std::vector<hipEvent_t> ev_lvl;
    std::vector<char> lvl_pending;
    // dist_overlap, per partitioned level l: its restricted rhs ghosts are
    // being exchanged on the side stream (the level-1 rhs after the cross pass,
    // behind the norm's host round trip); ev_rhs[l] marks the end
    std::vector<hipEvent_t> ev_rhs;
    std::vector<char> rhs_pending;
};

// the effective dist_overlap of a context (-1: by transport)
static long overlap_mode(const Dist *d) {
    if (g_dist_overlap >= 0) return g_dist_overlap;
    return d->comm ? 1 : 0;
}

void dist_free(mgx_ctx *c) {
    Dist *d = c->dist;
    if (!d) return;
    if (d->xs) (void)hipStreamSynchronize(d->xs);   // an early exchange may still run
    for (auto &p : d->parts) {
        for (auto &L : p.lv) {
            (void)hipFree(L.u[0]);
            (void)hipFree(L.u[1]);
            (void)hipFree(L.u[2]);
            (void)hipFree(L.rhs);
            (void)hipFree(L.v1);
            (void)hipFree(L.v2);
            for (double *f : {L.sa1, L.sb1, L.sa2, L.sb2}) (void)hipFree(f);
        }
        if (p.sub) free_ctx(p.sub);
        (void)hipFree(p.vga);
        (void)hipFree(p.dsum);
        (void)hipFree(p.partials);
    }
    if (d->comm) (void)ncclCommDestroy(d->comm);
    if (d->ev_comm) (void)hipEventDestroy(d->ev_comm);
    if (d->xs) (void)hipStreamDestroy(d->xs);
    if (d->ev_fork) (void)hipEventDestroy(d->ev_fork);
    if (d->ev_join) (void)hipEventDestroy(d->ev_join);
    for (hipEvent_t e : d->ev_lvl)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : d->ev_rhs)
        if (e) (void)hipEventDestroy(e);
    if (d->hsum) (void)hipHostFree(d->hsum);
    (void)hipFree(d->dsum_all);
    delete d;
    c->dist = nullptr;
}

static int build_dist(mgx_ctx *c, int world, const std::vector<int> &ranks) {
    Dist *d = c->dist;
    d->world = world;
    d->la = plan_la(c->N, c->L, world);
    for (int l = 0; l < d->la; ++l) CHK(plan_check(c->N, l, world));
    HIPCHK(hipHostMalloc(&d->hsum, sizeof(double) * 8));
    HIPCHK(hipMalloc(&d->dsum_all, sizeof(double) * 8));
    // the zero row the marches read for zero velocity rows: the finest pitch
    (void)hipFree(c->zrow);
    c->zrow = nullptr;
    HIPCHK(hipMalloc(&c->zrow, sizeof(double) * mgx::tower_pitch(c->N)));
    HIPCHK(hipMemsetAsync(c->zrow, 0, sizeof(double) * mgx::tower_pitch(c->N), c->stream));
    HIPCHK(hipStreamCreateWithFlags(&d->xs, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&d->ev_fork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&d->ev_join, hipEventDisableTiming));
    d->early_buf.assign(d->la, -1);
    d->lvl_pending.assign(d->la, 0);
    d->ev_lvl.assign(d->la, nullptr);
    for (auto &e : d->ev_lvl) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    d->rhs_pending.assign(d->la, 0);
    d->ev_rhs.assign(d->la, nullptr);
    for (auto &e : d->ev_rhs) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&d->ev_comm, hipEventDisableTiming));
    for (int r : ranks) {
        Part p;
        p.rank = r;
        double h = 1.0 / c->N;
        for (int l = 0; l < d->la; ++l) {
            PLevel L;
            L.n = c->N >> l;
            L.pitch = mgx::tower_pitch(L.n);
            L.coef = mgx::make_coef(c->dt, c->nu, h, c->opt.fp_mode == MGX_FP_FMA);
            alloc_rows(c->N, l, world, r, &L.ra, &L.rb, &L.lo, &L.hi);
            const bool third = l == 0 && L.n >= kCrossMinN;
            double **bufs[6] = {&L.u[0], &L.u[1], &L.rhs, &L.v1, &L.v2, &L.u[2]};
            for (double **b : bufs) {
                if (b == &L.u[2] && !third) continue;
                HIPCHK(hipMalloc(b, L.bytes()));
                HIPCHK(hipMemsetAsync(*b, 0, L.bytes(), c->stream));
            }
            p.lv.push_back(L);
            h = 2 * h;
        }
        mgx_options so = c->opt;
        so.device = -1;
        CHK(create_ctx(&p.sub, c->N >> d->la, c->L - d->la, c->dt, c->nu, &so, c->stream));
        HIPCHK(hipMalloc(&p.dsum, sizeof(double) * 8));
        HIPCHK(hipMalloc(&p.partials, sizeof(double) * 2 * mgx::norm_partials_size()));
        d->parts.push_back(p);
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    return MGX_OK;
}

// ---------------------------------------------------------------- transport
// Virtual ranks: all the row-block copies of one exchange (every part's ghost
// rows to both neighbours, or the all-gather of the replicated level's rhs)
// as ONE kernel instead of one blit launch per copy (G = 8: 14 per ghost
// exchange, 56 per all-gather).  Workgroup b copies chunk b - first[k] of
// copy k, 16 B per lane (the copies are whole pitched rows: 16-double
// multiples, 128-B aligned).
constexpr int kMaxCopies = 64;
constexpr long kCopyChunk = 8192;   // doubles per workgroup
struct CopyList {
    const double *src[kMaxCopies];
    double *dst[kMaxCopies];
    long cnt[kMaxCopies];
    int first[kMaxCopies + 1];   // prefix workgroup counts
    int n;
};

__global__ __launch_bounds__(256) void k_copy_list(const CopyList L) {
    const int b = blockIdx.x;
    int k = 0;
    while (k + 1 < L.n && b >= L.first[k + 1]) ++k;
    const long i0 = (long)(b - L.first[k]) * kCopyChunk;
    const long i1 = min(i0 + kCopyChunk, L.cnt[k]);
    const double2 *src = reinterpret_cast<const double2 *>(L.src[k]);
    double2 *dst = reinterpret_cast<double2 *>(L.dst[k]);
    for (long i = i0 / 2 + threadIdx.x; i < i1 / 2; i += 256) dst[i] = src[i];
}

struct CopyBatch {
    CopyList L{};
    int blocks = 0;
    int add(const double *src, double *dst, long cnt, hipStream_t st) {
        if (cnt <= 0) return MGX_OK;
        if ((cnt & 1) || ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15))
            return fail(MGX_E_INTERNAL, "copy list: rows not 16-B aligned");
        if (L.n == kMaxCopies) CHK(flush(st));
        L.src[L.n] = src;
        L.dst[L.n] = dst;
        L.cnt[L.n] = cnt;
        L.first[L.n] = blocks;
        blocks += (int)((cnt + kCopyChunk - 1) / kCopyChunk);
        L.first[++L.n] = blocks;
        return MGX_OK;
    }
    int flush(hipStream_t st) {
        if (L.n == 0) return MGX_OK;
        hipLaunchKernelGGL(k_copy_list, dim3((unsigned)blocks), dim3(256), 0, st, L);
        HIPCHK(hipGetLastError());
        L.n = 0;
        blocks = 0;
        return MGX_OK;
    }
};

// Virtual ranks: the parts' partial sums of squares added in part order (the
// host loop's order: bitwise the same) on the device, one read-back.
struct PtrList {
    const double *p[kMaxCopies];
    int n;
    int cont;   // continue the sum in *out (more than kMaxCopies parts)
};
__global__ void k_sum_list(const PtrList L, double *out) {
    if (threadIdx.x == 0) {
        double t = L.cont ? *out : 0.0;
        for (int i = 0; i < L.n; ++i) t += *L.p[i];
        *out = t;
    }
}

enum Field { kU, kRhs, kV1, kV2 };

static double *field(const PLevel &L, Field f, int buf = -1) {
    switch (f) {
        case kU: return buf >= 0 ? L.F(L.u[buf]) : L.U();
        case kRhs: return L.F(L.rhs);
        case kV1: return L.F(L.v1);
        default: return L.F(L.v2);
    }
}

// Refresh the ghost rows of the listed (level, field)s from the neighbouring
// ranks; over RCCL all of them go in ONE group (one latency, not one each).
struct XF {
    int l;
    Field f;
    int buf = -1;   // kU: this u buffer instead of the current one
};

// Issue one RCCL operation (a group, a collective) of this rank on stream st,
// chained after the rank's previous one: if that was issued on another stream,
// st first waits for its end (ev_comm).  Host issue order is the program order,
// the same on every rank, so the ranks' operations pair up in order and no two
// of one rank ever run at once -- whichever stream each was issued on.
template <class F>
static int comm_op(Dist *d, hipStream_t st, F &&issue) {
    if (g_dist_comm_chain && d->comm_last && d->comm_last != st)
        HIPCHK(hipStreamWaitEvent(st, d->ev_comm, 0));
    CHK(issue());
    HIPCHK(hipEventRecord(d->ev_comm, st));
    d->comm_last = st;
    return MGX_OK;
}

static int exchange_rows(mgx_ctx *c, const std::vector<XF> &xs, hipStream_t st) {
    Dist *d = c->dist;
    std::vector<Xfer> plan;
    if (d->local) {
        // part i's send to j lands where j's plan receives from i (the plan is
        // checked pairwise at context creation: plan_check); all of them in
        // one copy kernel (CopyBatch)
        CopyBatch cb;
        for (const XF &x : xs)
            for (size_t i = 0; i < d->parts.size(); ++i) {
                const PLevel &L = d->parts[i].lv[x.l];
                const long P = L.pitch;
                ghost_plan(c->N, x.l, d->world, d->parts[i].rank, plan);
                for (const Xfer &t : plan) {
                    PLevel &R = d->parts[t.peer].lv[x.l];
                    CHK(cb.add(field(L, x.f, x.buf) + (long)t.send_row * P,
                               field(R, x.f, x.buf) + (long)t.send_row * P,
                               (long)t.send_rows * P, st));
                }
            }
        return cb.flush(st);
    }
    Part &p = d->parts[0];
    if (!d->comm) return fail(MGX_E_INTERNAL, "ghost exchange: no communicator");
    return comm_op(d, st, [&]() -> int {
        ncclResult_t r = ncclGroupStart();
        for (const XF &x : xs) {
            PLevel &L = p.lv[x.l];
            const long P = L.pitch;
            double *a = field(L, x.f, x.buf);
            ghost_plan(c->N, x.l, d->world, p.rank, plan);
            for (const Xfer &t : plan) {
                if (r != ncclSuccess) break;
                r = ncclSend(a + (long)t.send_row * P, (size_t)t.send_rows * P, ncclDouble,
                             t.peer, d->comm, st);
                if (r == ncclSuccess)
                    r = ncclRecv(a + (long)t.recv_row * P, (size_t)t.recv_rows * P, ncclDouble,
                                 t.peer, d->comm, st);
            }
        }
        const ncclResult_t re = ncclGroupEnd();   // always close the group
        if (r == ncclSuccess) r = re;
        if (r != ncclSuccess)
            return fail(MGX_E_RCCL, std::string("ghost exchange: ") + ncclGetErrorString(r));
        return MGX_OK;
    });
}

// bytes moved by the parts this process holds: every row sent is read once
// and written once
static double halo_bytes(mgx_ctx *c, const std::vector<XF> &xs) {
    double bytes = 0;
    std::vector<Xfer> plan;
    for (const XF &x : xs)
        for (const Part &p : c->dist->parts) {
            ghost_plan(c->N, x.l, c->dist->world, p.rank, plan);
            for (const Xfer &t : plan) bytes += 16.0 * t.send_rows * p.lv[x.l].pitch;
        }
    return bytes;
}

static int xchg(mgx_ctx *c, const std::vector<XF> &xs) {
    if (c->dist->world == 1 || xs.size() == 0) return MGX_OK;
    int rc = MGX_OK;
    CHK(launch(c, MGX_K_HALO, xs.begin()->l, halo_bytes(c, xs),
               [&] { rc = exchange_rows(c, xs, c->stream); }));
    return rc;
}

static int xchg(mgx_ctx *c, int l, Field f) { return xchg(c, std::vector<XF>{XF{l, f}}); }

// All of the side stream's work is joined into the compute stream (dist_overlap).
static int settle(mgx_ctx *c) {
    Dist *d = c->dist;
    if (!d->early_pending) return MGX_OK;
    HIPCHK(hipStreamWaitEvent(c->stream, d->ev_join, 0));
    d->early_pending = false;
    std::fill(d->lvl_pending.begin(), d->lvl_pending.end(), 0);
    std::fill(d->rhs_pending.begin(), d->rhs_pending.end(), 0);
    return MGX_OK;
}

// Records the side stream's exchange like a launch (launch() times c->stream);
// ev_join (and ev_extra) mark its end.  Stream order on the side stream: a
// later wait on ev_join covers every earlier side exchange too.
template <class F>
static int side_exchange(mgx_ctx *c, const std::vector<XF> &xs, F &&post,
                         hipEvent_t ev_extra = nullptr) {
    Dist *d = c->dist;
    // (virtual ranks, dist_local_side 0: the same schedule on the compute stream)
    hipStream_t st = d->local && !g_dist_local_side ? c->stream : d->xs;
    if (st != c->stream) {
        HIPCHK(hipEventRecord(d->ev_fork, c->stream));
        HIPCHK(hipStreamWaitEvent(st, d->ev_fork, 0));
    }
    const bool rec = c->prof == 1 || c->prof == 2;
    hipEvent_t e0 = rec ? take_event(c) : nullptr, e1 = rec ? take_event(c) : nullptr;
    if (e0) HIPCHK(hipEventRecord(e0, st));
    CHK(exchange_rows(c, xs, st));
    if (e0 && e1) {
        HIPCHK(hipEventRecord(e1, st));
        const double b = halo_bytes(c, xs);
        c->pending.push_back({MGX_K_HALO, 0, b, b, e0, e1});
    }
    HIPCHK(hipEventRecord(d->ev_join, st));
    if (ev_extra) HIPCHK(hipEventRecord(ev_extra, st));
    d->early_pending = true;
    post();
    return MGX_OK;
}

// dist_overlap: the u ghost rows of buffer b of partitioned level l, just
// written by the level's pre-smoothing pass (or the finest level's cross
// pass) and next read by the level's post-smoothing pass after the coarser
// levels, exchanged on the side stream now -- behind the coarse part of the
// V-cycle instead of in front of the post pass.
static int early_u(mgx_ctx *c, int l, int b) {
    Dist *d = c->dist;
    if (overlap_mode(d) == 0 || d->world == 1 || l >= d->la) return MGX_OK;
    return side_exchange(
        c, {XF{l, kU, b}},
        [&] {
            d->lvl_pending[l] = 1;
            d->early_buf[l] = b;
        },
        d->ev_lvl[l]);
}

// Whether the current u buffer of level l has its ghost rows exchanged
// already (early_u); the compute stream waits for that exchange.  Consumes
// the state.
static int take_fresh(mgx_ctx *c, int l, bool *fresh) {
    Dist *d = c->dist;
    *fresh = false;
    if (l >= d->la) return MGX_OK;
    if (d->lvl_pending[l]) {
        HIPCHK(hipStreamWaitEvent(c->stream, d->ev_lvl[l], 0));
        d->lvl_pending[l] = 0;
    }
    *fresh = d->early_buf[l] >= 0 && !d->parts.empty() &&
             d->early_buf[l] == d->parts[0].lv[l].cur;
    d->early_buf[l] = -1;
    return MGX_OK;
}

// The compute stream waits for a side-stream exchange of level l's rhs ghosts
// (rhs_side), if one is pending.
static int take_rhs(mgx_ctx *c, int l) {
    Dist *d = c->dist;
    if (l < d->la && d->rhs_pending[l]) {
        HIPCHK(hipStreamWaitEvent(c->stream, d->ev_rhs[l], 0));
        d->rhs_pending[l] = 0;
    }
    return MGX_OK;
}

// Restricted rhs of the first replicated level: every rank wrote its own rows
// of the full array in its sub-context; make them whole everywhere.
static int gather_rhs(mgx_ctx *c) {
    Dist *d = c->dist;
    if (d->world > 1) {
        long row0, q;
        if (d->local) {
            CopyBatch cb;
            for (auto &dst : d->parts)
                for (auto &src : d->parts) {
                    if (&dst == &src) continue;
                    gather_rows(c->N, d->la, d->world, src.rank, &row0, &q);
                    const long P = dst.sub->lv[0].pitch, off = row0 * P;
                    CHK(cb.add(src.sub->lv[0].rhs + off, dst.sub->lv[0].rhs + off, q * P,
                               c->stream));
                }
            CHK(cb.flush(c->stream));
        } else {
            Part &p = d->parts[0];
            gather_rows(c->N, d->la, d->world, p.rank, &row0, &q);
            const long P = p.sub->lv[0].pitch;
            double *rhs = p.sub->lv[0].rhs;
            // in place: the send buffer is the receive buffer + rank * count
            CHK(comm_op(d, c->stream, [&]() -> int {
                NCCLCHK(ncclAllGather(rhs + row0 * P, rhs, (size_t)q * P, ncclDouble, d->comm,
                                      c->stream));
                return MGX_OK;
            }));
        }
    }
    for (auto &p : d->parts) p.sub->lv[0].zero = true;   // u[la] = 0 (multigrid.cpp:77)
    return MGX_OK;
}

// Sum the ranks' partial sums of squares -> norm on the host, in two halves:
// norm_issue enqueues the sum (all-reduce) and its read-back on the compute
// stream, norm_finish waits for it.  The cross pass issues its norm BEFORE the
// exchanges that follow it, so those run behind the host round trip instead of
// in front of the all-reduce (comm_op orders them after it).
static int norm_issue(mgx_ctx *c) {
    Dist *d = c->dist;
    if (d->local) {
        PtrList pl{};
        for (size_t i = 0; i < d->parts.size(); ++i) {
            pl.p[pl.n++] = d->parts[i].dsum;
            if (pl.n == kMaxCopies || i + 1 == d->parts.size()) {
                hipLaunchKernelGGL(k_sum_list, dim3(1), dim3(64), 0, c->stream, pl, d->dsum_all);
                HIPCHK(hipGetLastError());
                pl.n = 0;
                pl.cont = 1;
            }
        }
        HIPCHK(hipMemcpyAsync(d->hsum, d->dsum_all, sizeof(double), hipMemcpyDeviceToHost,
                              c->stream));
    } else {
        Part &p = d->parts[0];
        CHK(comm_op(d, c->stream, [&]() -> int {
            NCCLCHK(ncclAllReduce(p.dsum, p.dsum, 1, ncclDouble, ncclSum, d->comm, c->stream));
            return MGX_OK;
        }));
        HIPCHK(hipMemcpyAsync(d->hsum, p.dsum, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    }
    return MGX_OK;
}

static int norm_finish(mgx_ctx *c, double *norm) {
    HIPCHK(hipStreamSynchronize(c->stream));
    *norm = std::sqrt(c->dist->hsum[0]);
    return MGX_OK;
}

static int reduce_norm(mgx_ctx *c, double *norm) {
    CHK(norm_issue(c));
    return norm_finish(c, norm);
}

// ---------------------------------------------------------------- V-cycle
static mgx::SmoothArgs args_for(const PLevel &L) {
    mgx::SmoothArgs A{};
    A.uin = L.U();
    A.uout = L.F(L.u[L.nxt()]);
    A.rhs = L.F(L.rhs);
    A.v1 = L.F(L.v1);
    A.v2 = L.F(L.v2);
    A.n = L.n;
    A.pitch = L.pitch;
    A.c = L.coef;
    A.ra = L.ra;
    A.rb = L.rb;
    A.lo = L.lo;
    A.hi = L.hi;
    return A;
}

// Communication-avoiding post-smoothing: when a level's post-smoothing is ONE
// pass (nsmooth <= fuse), a coarse level's post pass also computes the
// kPostExt rows past each end of its block -- exactly what the neighbours
// compute there (same inputs, same operations: bitwise), from its 16 ghost
// rows of u_pre and rhs -- so the finer level's prolongation reads its own
// copy and the corrected u is never exchanged: one RCCL group per coarse
// level and cycle off the critical path (the u_pre ghosts before the pass
// stay, on the side stream with dist_overlap).
static bool post_ca(const mgx_ctx *c) {
    const int fuse = std::max(1, std::min(c->opt.fuse, mgx::kSmoothMaxSweeps));
    return c->opt.nsmooth >= 1 && c->opt.nsmooth <= fuse &&
           kPostExt + 2 * c->opt.nsmooth <= mgxplan::kGhost;
}

// nsmooth sweeps on partitioned level l in passes of <= fuse sweeps; the
// first pass may add the prolongation, the last may restrict or take the norm.
static int smooth(mgx_ctx *c, int l, bool prolong, bool restrict_, bool norm) {
    Dist *d = c->dist;
    const int sweeps = c->opt.nsmooth;
    const int fuse = std::max(1, std::min(c->opt.fuse, mgx::kSmoothMaxSweeps));
    const bool ca = post_ca(c);
    bool fresh = false;   // u ghosts exchanged early (dist_overlap)
    CHK(take_fresh(c, l, &fresh));
    CHK(take_rhs(c, l));
    for (int done = 0; done < sweeps;) {
        const int k = std::min(sweeps - done, fuse);
        const bool first = done == 0, last = done + k == sweeps;
        const bool zero = d->parts[0].lv[l].zero;
        const bool pr = prolong && first && !zero;
        const bool rs = restrict_ && last;
        const bool nm = norm && last && !rs;
        const bool ufresh = fresh && first;
        // (the coarser level's u for the prolongation: its own rows past the
        // block, ca, or its ghost rows exchanged)
        if (!zero && pr && l + 1 < d->la && !ca)
            CHK(ufresh ? xchg(c, l + 1, kU) : xchg(c, {XF{l, kU}, XF{l + 1, kU}}));
        else if (!zero && !ufresh)
            CHK(xchg(c, l, kU));
        int mode = 0;
        if (zero) mode |= mgx::kModeZero;
        if (pr) mode |= mgx::kModeProlong;
        if (rs) mode |= mgx::kModeRestrict;
        if (nm) mode |= mgx::kModeNorm;
        for (auto &p : d->parts) {
            PLevel &L = p.lv[l];
            mgx::SmoothArgs A = args_for(L);
            if (pr && ca && l >= 1) {   // + kPostExt rows past each end
                A.ra = std::max(0, L.ra - kPostExt);
                A.rb = (int)std::min<long>(L.n + 1, (long)L.rb + kPostExt);
            }
            if (pr || rs) {
                if (l + 1 < d->la) {
                    PLevel &Cl = p.lv[l + 1];
                    A.uc = Cl.U();
                    A.rhsc = Cl.F(Cl.rhs);
                    A.pitchc = Cl.pitch;
                } else {
                    Level &Cl = p.sub->lv[0];
                    A.uc = Cl.U();
                    A.rhsc = Cl.rhs;
                    A.pitchc = Cl.pitch;
                }
            }
            A.partials = p.partials;
            A.norm_out = p.dsum;
            A.norm_sqrt = false;
            A.zrow = c->zrow;
            A.vz = L.vz;
            // velocity generated from level 0's factors (global rows and
            // columns; dist_upload / the row-block upload's vgen_rows)
            if (L.vgen && g_vgen && p.vga && p.lv[0].sb1) {
                A.vg.a = p.vga;
                A.vg.b1 = p.lv[0].sb1;
                A.vg.b2 = p.lv[0].sb2;
                A.vg.l = l;
                A.vg.strided = c->opt.tower_mode == MGX_TOWER_CORRECT ? 1 : 0;
            }
            const bool vgu = mgx::smooth_generates_velocity(A, k, mode);
            // points of the launched rows: the owned ones, or with the
            // communication-avoiding extension the kPostExt rows past each end
            const double M = double(A.rb - A.ra) * double(L.n + 1);
            double bytes = 40.0 * k * M;
            const double Mc = M / 4;
            if (pr) bytes += 32.0 * M + 8.0 * Mc;
            if (rs) bytes += 40.0 * M + 24.0 * Mc;
            if (nm) bytes += 48.0 * M;
            const double cbytes = 8.0 * ((zero ? 4.0 : 5.0) * M - (vgu ? 2.0 * M : 0.0) +
                                         ((pr ? 1 : 0) + (rs ? 1 : 0)) * Mc);
            int blocks = 0;
            CHK(launch(c, pr ? MGX_K_PSMOOTH : MGX_K_GS, l, bytes, cbytes,
                       [&] { blocks = mgx::launch_smooth(A, k, mode, c->stream); }));
            if (blocks < 0) return fail(MGX_E_ARG, "launch_smooth: unsupported sweeps/mode");
            L.cur = L.nxt();
            L.zero = false;
        }
        done += k;
    }
    return MGX_OK;
}

// rhs of level l+1 restricted (owned rows): refresh its ghosts, or gather it
// into the replicated sub-contexts; u[l+1] = 0 for the coming coarse solve
// side (dist_overlap >= 1, the cross pass): a partitioned level's rhs ghosts
// go on the side stream -- behind the norm's host round trip -- and the level's
// next pass waits for them (take_rhs).
static int coarse_rhs_ready(mgx_ctx *c, int l, bool side = false) {
    Dist *d = c->dist;
    if (l + 1 < d->la) {
        if (side && overlap_mode(d) != 0 && d->world > 1)
            CHK(side_exchange(
                c, {XF{l + 1, kRhs}}, [&] { d->rhs_pending[l + 1] = 1; }, d->ev_rhs[l + 1]));
        else
            CHK(xchg(c, l + 1, kRhs));
        for (auto &p : d->parts) p.lv[l + 1].zero = true;
        return MGX_OK;
    }
    return gather_rhs(c);
}

static int coarse_cycle(mgx_ctx *c, int l);

static int dist_level(mgx_ctx *c, int l, bool want_norm) {
    for (int sh = 0; sh < c->opt.shape; ++sh) {
        const bool last = sh == c->opt.shape - 1;
        CHK(smooth(c, l, false, /*restrict=*/true, false));
        CHK(coarse_rhs_ready(c, l));
        CHK(early_u(c, l, c->dist->parts[0].lv[l].cur));
        CHK(coarse_cycle(c, l + 1));
        CHK(smooth(c, l, /*prolong=*/true, false, want_norm && last));
    }
    return MGX_OK;
}

// the V-cycle below a partitioned level l-1: partitioned or replicated
static int coarse_cycle(mgx_ctx *c, int l) {
    Dist *d = c->dist;
    if (l < d->la) return dist_level(c, l, false);
    for (auto &p : d->parts) CHK(op_vcycle(p.sub, 0));
    return MGX_OK;
}

static bool dist_cross_ok(mgx_ctx *c) {
    Dist *d = c->dist;
    return cross_cycle_on() && d->la >= 1 && d->parts[0].lv[0].u[2] &&
           c->opt.smoother == 0 && c->opt.shape >= 1 &&
           (c->opt.nsmooth == 2 || c->opt.nsmooth == 3) && c->opt.fuse >= c->opt.nsmooth;
}

static void dist_drop_spec(mgx_ctx *c) {
    for (auto &p : c->dist->parts)
        if (!p.lv.empty()) p.lv[0].spec = -1;
}

// Cross-cycle pass on the row blocks of level 0 (mgx.hip:op_cross): u ghosts
// (16 rows: the pass's cone is 14) and, if level 1 is partitioned, its u
// ghosts for the prolongation; afterwards the restricted rhs of the next cycle
// is made ready on level 1 and the per-rank norm sums are reduced by the caller.
//
// dist_overlap >= 1: the level-0 ghosts were exchanged on the side stream
// right after the pass that wrote them (early_u), behind the coarse levels;
// only level 1's u ghosts remain.  dist_overlap = 2: those go on the second
// stream too (forked after the work that produced the sent rows) while the
// compute stream runs the pass's unguarded interior march over rows
// [ra+16, rb-16) -- whose cone [ra+2, rb-2) and coarse parents are all owned,
// so it needs no ghost row -- and the pass's edge launch, which the split pass
// always has (boundary strips, global bands), takes the two 16-row bands next
// to the ghosts too, after the join (launch_xsmooth phases 1 and 2).
// Outputs, u_pre / u_post / coarse rhs, are the same rows either way: bitwise.
static int dist_cross(mgx_ctx *c, bool store_post, bool norm) {
    Dist *d = c->dist;
    const int G = kGhostFine;
    const int k = c->opt.nsmooth;
    // u ghosts of level 0 (unless exchanged early, dist_overlap) and of level 1
    bool fresh = false;
    CHK(take_fresh(c, 0, &fresh));
    std::vector<XF> xl;
    if (!fresh) xl.push_back(XF{0, kU});
    if (1 < d->la && !post_ca(c)) xl.push_back(XF{1, kU});
    // (the split launches are the unguarded kernel's: xfast on, d > 0)
    bool ov = overlap_mode(d) == 2 && d->world > 1 && !xl.empty() && mgx::get_xfast() != 0;
    for (auto &p : d->parts) ov = ov && p.lv[0].rb - p.lv[0].ra >= 4 * G && p.lv[0].coef.dgs > 0;
    if (ov)
        CHK(side_exchange(c, xl, [] {}));
    else if (!xl.empty())
        CHK(xchg(c, xl));
    // one launch (phase 1 / 2) or both of the pass over owned rows [ra, rb) of
    // part p; an MGX status, the norm partials written in *blocks_out
    auto pass = [&](Part &p, int P, int Q, int phase, int done, int *blocks_out) -> int {
        PLevel &L = p.lv[0];
        mgx::XArgs A;
        A.uin = L.U();
        A.upost = L.F(L.u[P]);
        A.upre = L.F(L.u[Q]);
        A.rhs = L.F(L.rhs);
        A.v1 = L.F(L.v1);
        A.v2 = L.F(L.v2);
        if (1 < d->la) {
            PLevel &Cl = p.lv[1];
            A.uc = Cl.U();
            A.rhsc = Cl.F(Cl.rhs);
            A.pitchc = Cl.pitch;
        } else {
            Level &Cl = p.sub->lv[0];
            A.uc = Cl.U();
            A.rhsc = Cl.rhs;
            A.pitchc = Cl.pitch;
        }
        const double Mown = L.Mown(), Mc = Mown / 4;
        A.partials = p.partials;
        A.norm_out = p.dsum;
        A.norm_sqrt = false;
        A.n = L.n;
        A.pitch = L.pitch;
        A.c = L.coef;
        A.store_post = store_post;
        A.sa1 = L.sa1;
        A.sb1 = L.sb1;
        A.sa2 = L.sa2;
        A.sb2 = L.sb2;
        A.ra = L.ra;
        A.rb = L.rb;
        A.lo = L.lo;
        A.hi = L.hi;
        A.band = phase ? G : 0;
        A.phase = phase;
        A.partials_done = done;
        // (a split pass's bytes and time are counted on its second launch)
        const double bytes =
            phase == 1 ? 0.0 : (32.0 + 40.0 * k + 48.0 + 40.0 * k + 40.0) * Mown + 32.0 * Mc;
        const double cbytes =
            phase == 1 ? 0.0
                       : 8.0 * ((store_post ? 6.0 : 5.0) * Mown - (L.sa1 ? 2.0 * Mown : 0.0) +
                                2.0 * Mc);
        int blocks = 0;
        if (phase == 0) {
            CHK(launch(c, MGX_K_XSMOOTH, 0, bytes, cbytes,
                       [&] { blocks = mgx::launch_xsmooth(A, k, c->stream); }));
        } else {   // a split pass is timed from its first launch to its second
            const bool rec = c->prof == 1 || c->prof == 2;
            hipEvent_t &e0 = p.xe0;
            if (phase == 1) e0 = rec ? take_event(c) : nullptr;
            if (phase == 1 && e0) HIPCHK(hipEventRecord(e0, c->stream));
            blocks = mgx::launch_xsmooth(A, k, c->stream);
            CHK(check_launch("launch_xsmooth"));
            hipEvent_t e1 = (phase == 2 && e0) ? take_event(c) : nullptr;
            if (e1) {
                HIPCHK(hipEventRecord(e1, c->stream));
                c->pending.push_back({MGX_K_XSMOOTH, 0, bytes, cbytes, e0, e1});
                e0 = nullptr;
            }
        }
        if (blocks < 0) return fail(MGX_E_ARG, "launch_xsmooth: unsupported sweeps / block");
        *blocks_out = blocks;
        return MGX_OK;
    };
    std::vector<std::pair<int, int>> bufs;
    for (auto &p : d->parts) {
        PLevel &L = p.lv[0];
        int P = -1, Q = -1;
        for (int i = 0; i < 3; ++i)
            if (i != L.cur) (P < 0 ? P : Q) = i;
        bufs.push_back({P, Q});
    }
    if (!ov) {
        for (size_t i = 0; i < d->parts.size(); ++i) {
            int blocks = 0;
            CHK(pass(d->parts[i], bufs[i].first, bufs[i].second, 0, 0, &blocks));
        }
    } else {
        std::vector<int> done(d->parts.size(), 0);
        for (size_t i = 0; i < d->parts.size(); ++i)
            CHK(pass(d->parts[i], bufs[i].first, bufs[i].second, 1, 0, &done[i]));
        HIPCHK(hipStreamWaitEvent(c->stream, d->ev_join, 0));
        for (size_t i = 0; i < d->parts.size(); ++i) {
            int blocks = 0;
            CHK(pass(d->parts[i], bufs[i].first, bufs[i].second, 2, done[i], &blocks));
        }
    }
    for (size_t i = 0; i < d->parts.size(); ++i) {
        PLevel &L = d->parts[i].lv[0];
        L.xin = L.cur;
        L.cur = bufs[i].first;
        L.spec = bufs[i].second;
        L.zero = false;
    }
    // the norm first: its all-reduce and read-back are what the host waits
    // for; the exchanges below run behind that round trip (dist_overlap)
    if (norm) CHK(norm_issue(c));
    CHK(coarse_rhs_ready(c, 0, /*side=*/true));
    // the next cycle's level-0 input is u_pre: its ghosts now, on the side
    // stream, behind the coarse levels (after the coarse rhs exchange, which
    // the next level needs first)
    return early_u(c, 0, d->parts[0].lv[0].spec);
}

bool dist_post_predictable(mgx_ctx *c) {
    Dist *d = c->dist;
    return d->la >= 1 && dist_cross_ok(c);
}

// The last cross pass did not store u_post (mgx.hip:op_redo_post): prolongation
// + post-smoothing of each row block from the pass's input and the untouched
// level-1 correction, bitwise the pass's u_post (the unfused schedule).
int dist_redo_post(mgx_ctx *c) {
    Dist *d = c->dist;
    HIPCHK(hipSetDevice(c->device));
    for (auto &p : d->parts) {
        PLevel &L = p.lv[0];
        if (L.xin < 0) return fail(MGX_E_INTERNAL, "redo post-smoothing: no cross pass input");
        L.cur = L.xin;
        L.spec = -1;
        L.zero = false;
        if (1 < d->la)
            p.lv[1].zero = false;   // u[1] still holds the correction
        else
            p.sub->lv[0].zero = false;
    }
    return smooth(c, 0, /*prolong=*/true, false, false);
}

int dist_vcycle(mgx_ctx *c, double *norm, bool store_post) {
    Dist *d = c->dist;
    HIPCHK(hipSetDevice(c->device));
    if (d->la == 0) {   // everything replicated
        for (auto &p : d->parts) CHK(op_vcycle(p.sub, 0, norm, store_post));
        return MGX_OK;
    }
    if (norm && dist_cross_ok(c)) {
        if (d->parts[0].lv[0].spec >= 0) {   // pre-smoothing + restriction done
            for (auto &p : d->parts) {
                p.lv[0].cur = p.lv[0].spec;
                p.lv[0].spec = -1;
            }
        } else {
            CHK(smooth(c, 0, false, /*restrict=*/true, false));
            CHK(coarse_rhs_ready(c, 0));
            CHK(early_u(c, 0, d->parts[0].lv[0].cur));
        }
        // W-cycles: visit sh's post- and visit sh+1's pre-smoothing as one
        // cross pass (mgx.hip:op_vcycle)
        for (int sh = 1; sh < c->opt.shape; ++sh) {
            CHK(coarse_cycle(c, 1));
            CHK(dist_cross(c, /*store_post=*/false, /*norm=*/false));
            for (auto &p : d->parts) {
                p.lv[0].cur = p.lv[0].spec;
                p.lv[0].spec = -1;
            }
        }
        CHK(coarse_cycle(c, 1));
        if (c->post_only) {   // mg_outer's last cycle: post-smoothing + norm only
            CHK(smooth(c, 0, /*prolong=*/true, false, /*norm=*/true));
            dist_drop_spec(c);
            return reduce_norm(c, norm);
        }
        CHK(dist_cross(c, store_post, /*norm=*/true));
        return norm_finish(c, norm);
    }
    dist_drop_spec(c);
    CHK(dist_level(c, 0, norm != nullptr));
    if (norm) CHK(reduce_norm(c, norm));
    return MGX_OK;
}

int dist_residual_norm(mgx_ctx *c, double *norm) {
    Dist *d = c->dist;
    HIPCHK(hipSetDevice(c->device));
    CHK(settle(c));
    if (d->la == 0) {
        for (auto &p : d->parts) CHK(op_residual_norm(p.sub, 0, norm));
        return MGX_OK;
    }
    CHK(xchg(c, 0, kU));
    for (auto &p : d->parts) {
        PLevel &L = p.lv[0];
        CHK(launch(c, MGX_K_RESNORM, 0, 48.0 * L.Mown(), 32.0 * L.Mown(), [&] {
            mgx::launch_residual_norm(L.U(), L.F(L.rhs), L.F(L.v1), L.F(L.v2), L.n, L.pitch,
                                      L.coef, p.partials, p.dsum, c->stream, L.ra, L.rb,
                                      /*take_sqrt=*/false);
        }));
    }
    return reduce_norm(c, norm);
}

int dist_rhs(mgx_ctx *c) {
    Dist *d = c->dist;
    HIPCHK(hipSetDevice(c->device));
    CHK(settle(c));
    dist_drop_spec(c);
    if (d->la == 0) {
        for (auto &p : d->parts) CHK(op_rhs(p.sub));
        return MGX_OK;
    }
    CHK(xchg(c, 0, kU));
    for (auto &p : d->parts) {
        PLevel &L = p.lv[0];
        CHK(launch(c, MGX_K_RHS, 0, 32.0 * L.Mown(), [&] {
            mgx::launch_rhs(L.F(L.rhs), L.U(), L.F(L.v1), L.F(L.v2), L.n, L.pitch, L.coef,
                            c->stream, L.ra, L.rb);
        }));
    }
    return xchg(c, 0, kRhs);
}

// compute_rhs + the initial residual norm of mg_outer in one pass per part
// (mgx.hip:op_rhs_norm): u ghosts once, the rhs ghosts after
int dist_rhs_norm(mgx_ctx *c, double *res0) {
    Dist *d = c->dist;
    HIPCHK(hipSetDevice(c->device));
    CHK(settle(c));
    dist_drop_spec(c);
    if (d->la == 0) {
        CHK(dist_rhs(c));
        return dist_residual_norm(c, res0);
    }
    CHK(xchg(c, 0, kU));
    for (auto &p : d->parts) {
        PLevel &L = p.lv[0];
        CHK(launch(c, MGX_K_RHS, 0, 80.0 * L.Mown(), 32.0 * L.Mown(), [&] {
            mgx::launch_rhs_norm(L.F(L.rhs), L.U(), L.F(L.v1), L.F(L.v2), L.n, L.pitch, L.coef,
                                 p.partials, p.dsum, c->stream, L.ra, L.rb,
                                 /*take_sqrt=*/false);
        }));
    }
    CHK(xchg(c, 0, kRhs));
    return reduce_norm(c, res0);
}

// mgx_synchronize of a partitioned context: the side stream's pending
// exchanges are joined into the compute stream first, so that once the host
// has synchronised it, no RCCL operation of this rank is in flight (a caller's
// own collectives -- torch.distributed's barrier in bench.py -- may follow).
int dist_settle(mgx_ctx *c) { return settle(c); }

// mgx_velocity_factored of a partitioned context: its first part's levels
int dist_velocity_mask(mgx_ctx *c) {
    Dist *d = c->dist;
    if (d->parts.empty() || d->parts[0].lv.empty()) return 0;
    const Part &p = d->parts[0];
    int f = p.lv[0].sa1 ? 1 : 0;
    for (size_t l = 1; l < p.lv.size() && l < 31; ++l)
        if (p.lv[l].vgen && g_vgen) f |= 1 << l;
    return f;
}

int dist_nsub(mgx_ctx *c) { return c->dist ? (int)c->dist->parts.size() : 0; }
mgx_ctx *dist_sub(mgx_ctx *c, int i) { return c->dist->parts[i].sub; }
int dist_la(mgx_ctx *c) { return c->dist ? c->dist->la : c->L; }

// ---------------------------------------------------------------- data movement
// Level-0 velocity factors of a part: device copies of full-length arrays
// (row factors n+1, column factors pitch), from device (T's) or host vectors
// covering rows [row0, row0 + rows).
static void drop_factors(PLevel &L) {
    for (double **f : {&L.sa1, &L.sb1, &L.sa2, &L.sb2}) {
        (void)hipFree(*f);
        *f = nullptr;
    }
}
static int part_factors(PLevel &L, const double *a1, const double *b1, const double *a2,
                        const double *b2, long row0, long rows, hipMemcpyKind kind,
                        hipStream_t st) {
    drop_factors(L);
    const size_t ra = sizeof(double) * (size_t)(L.n + 1), rb = sizeof(double) * (size_t)L.pitch;
    HIPCHK(hipMalloc(&L.sa1, ra));
    HIPCHK(hipMalloc(&L.sa2, ra));
    HIPCHK(hipMalloc(&L.sb1, rb));
    HIPCHK(hipMalloc(&L.sb2, rb));
    for (double *f : {L.sa1, L.sa2}) HIPCHK(hipMemsetAsync(f, 0, ra, st));
    for (double *f : {L.sb1, L.sb2}) HIPCHK(hipMemsetAsync(f, 0, rb, st));
    const size_t na = sizeof(double) * (size_t)rows;
    const size_t nb = sizeof(double) * (size_t)(kind == hipMemcpyHostToDevice ? L.n + 1 : L.pitch);
    HIPCHK(hipMemcpyAsync(L.sa1 + row0, a1 + (kind == hipMemcpyHostToDevice ? 0 : row0), na, kind, st));
    HIPCHK(hipMemcpyAsync(L.sa2 + row0, a2 + (kind == hipMemcpyHostToDevice ? 0 : row0), na, kind, st));
    HIPCHK(hipMemcpyAsync(L.sb1, b1, nb, kind, st));
    HIPCHK(hipMemcpyAsync(L.sb2, b2, nb, kind, st));
    HIPCHK(hipStreamSynchronize(st));
    return MGX_OK;
}

// Build the full tower in a temporary single-GPU context (the reference
// construction, multigrid.cpp:148-160), then copy every rank's rows out of it.
int dist_upload(mgx_ctx *c, const double *u0, const double *v1, const double *v2,
                hipMemcpyKind kind) {
    Dist *d = c->dist;
    HIPCHK(hipSetDevice(c->device));
    CHK(settle(c));
    std::fill(d->early_buf.begin(), d->early_buf.end(), -1);
    mgx_options o = c->opt;
    o.device = -1;
    mgx_ctx *T = nullptr;
    CHK(create_ctx(&T, c->N, c->L, c->dt, c->nu, &o, c->stream));
    int rc = upload_ctx(T, u0, v1, v2, kind);
    for (auto &p : d->parts) {
        // the generated velocity of levels 1-2 (checked over the whole level in T)
        (void)hipFree(p.vga);
        p.vga = nullptr;
        if (rc == MGX_OK && T->vga) {
            const size_t vb = sizeof(double2) * (size_t)(c->N + 2);
            if (hipMalloc(&p.vga, vb) != hipSuccess ||
                hipMemcpyAsync(p.vga, T->vga, vb, hipMemcpyDeviceToDevice, c->stream) !=
                    hipSuccess)
                rc = fail(MGX_E_HIP, "dist_upload: vgen table");
        }
        for (int l = 0; rc == MGX_OK && l < d->la; ++l) {
            PLevel &L = p.lv[l];
            Level &F = T->lv[l];
            const size_t cnt = sizeof(double) * (size_t)(L.hi - L.lo + 1) * L.pitch;
            const long off = (long)L.lo * L.pitch;
            rc = hipMemcpyAsync(L.v1, F.v1 + off, cnt, hipMemcpyDeviceToDevice, c->stream) ||
                 hipMemcpyAsync(L.v2, F.v2 + off, cnt, hipMemcpyDeviceToDevice, c->stream);
            if (rc == MGX_OK && l == 0)
                rc = hipMemcpyAsync(L.u[0], F.U() + off, cnt, hipMemcpyDeviceToDevice, c->stream);
            if (rc == MGX_OK)
                rc = hipMemsetAsync(L.rhs, 0, cnt, c->stream) ||
                     (l > 0 ? hipMemsetAsync(L.u[0], 0, cnt, c->stream) : hipSuccess);
            if (rc) rc = fail(MGX_E_HIP, "dist_upload: copy");
            L.cur = 0;
            L.spec = -1;
            L.zero = false;
            L.vz = F.vz;
            L.vgen = F.vgen && p.vga;
            if (rc == MGX_OK && l == 0) {   // the whole level's velocity factors, if any
                if (F.sa1)
                    rc = part_factors(L, F.sa1, F.sb1, F.sa2, F.sb2, 0, L.n + 1,
                                      hipMemcpyDeviceToDevice, c->stream);
                else
                    drop_factors(L);
            }
        }
        for (int l = d->la; rc == MGX_OK && l < c->L; ++l) {
            Level &S = p.sub->lv[l - d->la];
            Level &F = T->lv[l];
            const size_t cnt = sizeof(double) * (size_t)(F.n + 1) * F.pitch;
            rc = hipMemcpyAsync(S.v1, F.v1, cnt, hipMemcpyDeviceToDevice, c->stream) ||
                 hipMemcpyAsync(S.v2, F.v2, cnt, hipMemcpyDeviceToDevice, c->stream);
            if (rc == MGX_OK && l == 0)
                rc = hipMemcpyAsync(S.u[0], F.U(), cnt, hipMemcpyDeviceToDevice, c->stream);
            if (rc) rc = fail(MGX_E_HIP, "dist_upload: copy");
            S.cur = 0;
            S.zero = false;
            S.vz = F.vz;
        }
    }
    if (rc == MGX_OK && hipStreamSynchronize(c->stream) != hipSuccess)
        rc = fail(MGX_E_HIP, "dist_upload: sync");
    free_ctx(T);
    return rc;
}

int dist_download(mgx_ctx *c, double *u, hipMemcpyKind kind) {
    Dist *d = c->dist;
    HIPCHK(hipSetDevice(c->device));
    CHK(settle(c));
    if (d->la == 0) {
        mgx_ctx *s = d->parts[0].sub;
        Level &L = s->lv[0];
        const size_t row = (L.n + 1) * sizeof(double);
        HIPCHK(hipMemcpy2DAsync(u, row, L.U(), L.pitch * sizeof(double), row, L.n + 1, kind,
                                c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        return MGX_OK;
    }
    const long n = c->N;
    const size_t row = (n + 1) * sizeof(double);
    if (d->local) {
        for (auto &p : d->parts) {
            PLevel &L = p.lv[0];
            HIPCHK(hipMemcpy2DAsync(u + (long)L.ra * (n + 1), row, L.U() + (long)L.ra * L.pitch,
                                    L.pitch * sizeof(double), row, L.rb - L.ra, kind, c->stream));
        }
        HIPCHK(hipStreamSynchronize(c->stream));
        return MGX_OK;
    }
    // RCCL: all-gather the owned blocks into a full temporary, then copy out
    Part &p = d->parts[0];
    PLevel &L = p.lv[0];
    const long P = L.pitch, q = n / d->world;
    double *full = nullptr;
    HIPCHK(hipMalloc(&full, sizeof(double) * (size_t)(n + 1) * P));
    int rc = MGX_OK;
    ncclResult_t r1 = ncclSuccess;
    rc = comm_op(d, c->stream, [&]() -> int {
        r1 = ncclAllGather(L.U() + (long)L.ra * P, full, (size_t)q * P, ncclDouble, d->comm,
                           c->stream);
        return MGX_OK;
    });
    if (rc) {
        (void)hipFree(full);
        return rc;
    }
    // Drain before the next enqueue: with a size-1 communicator, RCCL 2.27's
    // all-gather followed directly by further stream work segfaulted on the
    // host (tests/test_gpu_dist.py::test_rccl_world1_equals_single).  The
    // download is off the hot path, so the sync costs nothing that matters.
    if (r1 == ncclSuccess && hipStreamSynchronize(c->stream) != hipSuccess) {
        (void)hipFree(full);
        return fail(MGX_E_HIP, "dist_download: sync");
    }
    // row n (boundary) lives on the last rank
    if (r1 == ncclSuccess && p.rank == d->world - 1)
        (void)hipMemcpyAsync(full + n * P, L.U() + n * P, sizeof(double) * P,
                             hipMemcpyDeviceToDevice, c->stream);
    if (r1 == ncclSuccess)
        rc = comm_op(d, c->stream, [&]() -> int {
            r1 = ncclBroadcast(full + n * P, full + n * P, (size_t)P, ncclDouble, d->world - 1,
                               d->comm, c->stream);
            return MGX_OK;
        });
    if (r1 != ncclSuccess) rc = fail(MGX_E_RCCL, ncclGetErrorString(r1));
    if (rc == MGX_OK &&
        (hipMemcpy2DAsync(u, row, full, P * sizeof(double), row, n + 1, kind, c->stream) ||
         hipStreamSynchronize(c->stream)))
        rc = fail(MGX_E_HIP, "dist_download");
    (void)hipFree(full);
    return rc;
}

// Owned finest-level rows [ra, rb) of local part `part` (every rank owns a
// contiguous block; the last one also owns the boundary row n).
int dist_owned_rows(mgx_ctx *c, int part, int *ra, int *rb) {
    Dist *d = c->dist;
    if (part < 0 || part >= (int)d->parts.size()) return fail(MGX_E_ARG, "bad part");
    plan_rows(c->N, 0, d->world, d->parts[part].rank, ra, rb);
    return MGX_OK;
}

// Row-block download (the counterpart of the row-block upload: no rank ever
// holds the whole grid): the owned rows of one local part, reference layout
// ((rb-ra) x (N+1) doubles).  No communication.
int dist_download_rows(mgx_ctx *c, int part, double *out, hipMemcpyKind kind) {
    Dist *d = c->dist;
    HIPCHK(hipSetDevice(c->device));
    CHK(settle(c));
    int ra, rb;
    CHK(dist_owned_rows(c, part, &ra, &rb));
    const long n = c->N;
    const size_t row = (n + 1) * sizeof(double);
    const double *src;
    long P;
    if (d->la == 0) {   // everything replicated: the part's rows of its full copy
        Level &S = d->parts[part].sub->lv[0];
        src = S.U();
        P = S.pitch;
    } else {
        PLevel &L = d->parts[part].lv[0];
        src = L.U();
        P = L.pitch;
    }
    // (PLevel::U() is offset so that + r * pitch is global row r, like a full field)
    HIPCHK(hipMemcpy2DAsync(out, row, src + (long)ra * P, P * sizeof(double), row, rb - ra, kind,
                            c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MGX_OK;
}

// Row-block upload, correct tower: which partitioned coarse levels generate
// their velocity (PLevel::vgen) from the block's level-0 factors.  Level l's
// entry (i, j) is the finest (2^l i, 2^l j); the generator reads the row
// factor pair at finest row 2^l i, which for a coarse GHOST row lies outside
// the rows this rank factored -- its pair is the level's own exchanged entry
// in column j*/2^l (the finest row factors are the entries of column j*,
// where the column factor is exactly 1: sepvel.h), so it is filled from
// there.  Then every entry of every allocated row of the level is checked
// bit for bit against the generator (k_vgen_check): a level whose rows do not
// all match keeps reading its arrays.  Each rank decides for its own block.
static int vgen_rows(mgx_ctx *c) {
    Dist *d = c->dist;
    for (auto &p : d->parts) {
        PLevel &F = p.lv[0];
        for (size_t l = 1; l < p.lv.size(); ++l) p.lv[l].vgen = false;
        if (!p.vga || !F.sb1 || F.js1 < 0 || F.js2 < 0 || d->la < 2) continue;
        // fill every level first (a later level rewrites rows of an earlier
        // one with the same values on a consistent tower), then check
        for (int l = 1; l < d->la; ++l) {
            PLevel &L = p.lv[l];
            const long m = (1L << l) - 1;
            if ((F.js1 & m) || (F.js2 & m)) continue;
            mgx::launch_vgen_fill_rows(p.vga, L.F(L.v1), L.F(L.v2), L.pitch, l,
                                       (int)(F.js1 >> l), (int)(F.js2 >> l), L.lo, L.hi,
                                       c->stream);
            CHK(check_launch("vgen_fill_rows"));
        }
        int *dok = nullptr;
        HIPCHK(hipMalloc(&dok, sizeof(int) * d->la));
        std::vector<int> ok(d->la, 1);
        int rc = hipMemcpyAsync(dok, ok.data(), sizeof(int) * d->la, hipMemcpyHostToDevice,
                                c->stream) == hipSuccess ? MGX_OK : fail(MGX_E_HIP, "vgen_rows");
        for (int l = 1; l < d->la && rc == MGX_OK; ++l) {
            PLevel &L = p.lv[l];
            mgx::VGen g;
            g.a = p.vga;
            g.b1 = F.sb1;
            g.b2 = F.sb2;
            g.l = l;
            g.strided = 1;
            mgx::launch_vgen_check(L.F(L.v1), L.F(L.v2), L.n, L.pitch, g, dok + l, c->stream,
                                   L.lo, L.hi);
            rc = check_launch("vgen_check (rows)");
        }
        if (rc == MGX_OK &&
            (hipMemcpyAsync(ok.data(), dok, sizeof(int) * d->la, hipMemcpyDeviceToHost,
                            c->stream) != hipSuccess ||
             hipStreamSynchronize(c->stream) != hipSuccess))
            rc = fail(MGX_E_HIP, "vgen_rows");
        (void)hipFree(dok);
        CHK(rc);
        for (int l = 1; l < d->la; ++l) {
            const long m = (1L << l) - 1;
            p.lv[l].vgen = ok[l] == 1 && !(F.js1 & m) && !(F.js2 & m) && !(p.lv[l].n & 1) &&
                           (p.lv[l].n << l) == c->N;
        }
    }
    return MGX_OK;
}

// Row-block upload (no rank ever holds the whole grid): each part gets its
// allocated rows [lo, hi] of u0 / v1 / v2 from the host, and the velocity
// tower is built locally by injection (MGX_TOWER_CORRECT, each level from the
// one above: coarse row I <- fine row 2I is owned by the same rank since row
// blocks start at even rows), ghost rows exchanged per level; the first
// replicated level is all-gathered and the sub-contexts inject the rest.
// The boundary row n of v is never read by any operator and is not gathered.
static int dist_upload_rows_impl(mgx_ctx *c, const double *const *u0s,
                                 const double *const *v1s, const double *const *v2s) {
    Dist *d = c->dist;
    HIPCHK(hipSetDevice(c->device));
    CHK(settle(c));
    std::fill(d->early_buf.begin(), d->early_buf.end(), -1);
    if (c->opt.tower_mode != MGX_TOWER_CORRECT)
        return fail(MGX_E_ARG, "mgx_upload_rows: needs tower_mode MGX_TOWER_CORRECT (the "
                               "reference tower mixes rows of the whole grid)");
    if (d->la == 0) return fail(MGX_E_ARG, "mgx_upload_rows: no partitioned level, use mgx_upload");
    const long w = c->N + 1;
    for (size_t i = 0; i < d->parts.size(); ++i) {
        if (!u0s || !v1s || !v2s || !u0s[i] || !v1s[i] || !v2s[i])
            return fail(MGX_E_ARG, "mgx_upload_rows: null array");
        Part &p = d->parts[i];
        for (size_t l = 0; l < p.lv.size(); ++l) {
            PLevel &L = p.lv[l];
            for (double *b : {L.u[0], L.u[1], L.u[2], L.rhs})
                if (b) HIPCHK(hipMemsetAsync(b, 0, L.bytes(), c->stream));
            L.cur = 0;
            L.spec = -1;
            L.zero = false;
            L.vz = 0x7fffffff;
            L.vgen = false;   // (set by vgen_rows once the tower is built)
        }
        PLevel &L = p.lv[0];
        const size_t row = w * sizeof(double), rows = L.hi - L.lo + 1;
        // velocity factors of this block's rows (every rank decides for its own
        // block: the factors only have to reproduce the rows its passes read)
        std::vector<double> a1, b1, a2, b2;
        L.js1 = L.js2 = -1;
        (void)hipFree(p.vga);
        p.vga = nullptr;
        if (L.n >= kCrossMinN && c->L > 1 &&
            factor_velocity(v1s[i], v2s[i], c->N, L.lo, (long)rows, L.coef.h * 0.5, a1, b1, a2,
                            b2, &L.js1, &L.js2)) {
            CHK(part_factors(L, a1.data(), b1.data(), a2.data(), b2.data(), L.lo, (long)rows,
                             hipMemcpyHostToDevice, c->stream));
            // the generator's row-factor pairs (VGen::a) of this block's rows;
            // the coarse levels' ghost rows are added from their own exchanged
            // rows below (vgen_rows)
            std::vector<double2> h(rows);
            for (size_t k = 0; k < rows; ++k) h[k] = make_double2(a1[k], a2[k]);
            const size_t vb = sizeof(double2) * (size_t)(c->N + 2);
            HIPCHK(hipMalloc(&p.vga, vb));
            HIPCHK(hipMemsetAsync(p.vga, 0, vb, c->stream));
            HIPCHK(hipMemcpyAsync(p.vga + L.lo, h.data(), sizeof(double2) * rows,
                                  hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));   // h goes out of scope
        } else {
            drop_factors(L);
        }
        HIPCHK(hipMemcpy2DAsync(L.u[0], L.pitch * sizeof(double), u0s[i], row, row, rows,
                                hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpy2DAsync(L.v1, L.pitch * sizeof(double), v1s[i], row, row, rows,
                                hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpy2DAsync(L.v2, L.pitch * sizeof(double), v2s[i], row, row, rows,
                                hipMemcpyHostToDevice, c->stream));
    }
    // partitioned coarse levels: owned rows by injection, then ghost rows
    for (int l = 1; l < d->la; ++l) {
        for (auto &p : d->parts) {
            PLevel &F = p.lv[l - 1], &C = p.lv[l];
            for (int f = 0; f < 2; ++f) {
                double *dst = (f ? C.F(C.v2) : C.F(C.v1)) + (long)C.ra * C.pitch;
                const double *src = (f ? F.F(F.v2) : F.F(F.v1)) + 2L * C.ra * F.pitch;
                mgx::launch_injection_rows(dst, C.pitch, src, F.pitch, C.rb - C.ra, C.n + 1,
                                           c->stream);
                CHK(check_launch("tower injection (rows)"));
            }
        }
        CHK(xchg(c, {XF{l, kV1}, XF{l, kV2}}));
    }
    CHK(vgen_rows(c));
    // first replicated level: owned rows into each sub-context, all-gathered
    const long nl = c->N >> d->la, q = nl / d->world;
    for (auto &p : d->parts) {
        PLevel &F = p.lv[d->la - 1];
        Level &S = p.sub->lv[0];
        int ra, rb;
        plan_rows(c->N, d->la, d->world, p.rank, &ra, &rb);
        for (int f = 0; f < 2; ++f)
            mgx::launch_injection_rows((f ? S.v2 : S.v1) + (long)ra * S.pitch, S.pitch,
                                       (f ? F.F(F.v2) : F.F(F.v1)) + 2L * ra * F.pitch,
                                       F.pitch, std::min<long>(rb, nl) - ra, nl + 1, c->stream);
        CHK(check_launch("tower injection (replicated level)"));
        for (auto &L : p.sub->lv) {
            for (double *b : {L.u[0], L.u[1], L.rhs})
                HIPCHK(hipMemsetAsync(b, 0, sizeof(double) * L.pitch * (L.n + 1), c->stream));
            L.cur = 0;
            L.spec = -1;
            L.zero = false;
            L.vz = 0x7fffffff;   // the correct tower has no zero rows to skip
        }
    }
    if (d->world > 1) {
        for (int f = 0; f < 2; ++f) {
            if (d->local) {
                for (auto &dst : d->parts)
                    for (auto &src : d->parts) {
                        if (&dst == &src) continue;
                        Level &Sd = dst.sub->lv[0], &Ss = src.sub->lv[0];
                        const long off = (long)src.rank * q * Sd.pitch;
                        HIPCHK(hipMemcpyAsync((f ? Sd.v2 : Sd.v1) + off, (f ? Ss.v2 : Ss.v1) + off,
                                              sizeof(double) * q * Sd.pitch,
                                              hipMemcpyDeviceToDevice, c->stream));
                    }
            } else {
                Part &p = d->parts[0];
                Level &S = p.sub->lv[0];
                double *a = f ? S.v2 : S.v1;
                CHK(comm_op(d, c->stream, [&]() -> int {
                    NCCLCHK(ncclAllGather(a + (long)p.rank * q * S.pitch, a, (size_t)q * S.pitch,
                                          ncclDouble, d->comm, c->stream));
                    return MGX_OK;
                }));
            }
        }
    }
    for (auto &p : d->parts) CHK(build_tower(p.sub));   // correct mode: level by level
    HIPCHK(hipStreamSynchronize(c->stream));
    return MGX_OK;
}

static int create_dist_common(mgx_ctx **out, long n, int maxlvl, double dt, double nu,
                              const mgx_options *opt, mgx_ctx **cp) {
    mgx_options o;
    mgx_default_options(&o);
    if (opt) o = *opt;
    if (o.smoother != 0 || o.nsmooth < 1)
        return fail(MGX_E_ARG, "partitioned contexts need smoother 0 and nsmooth >= 1");
    // parent context: stream, scratch and options only; its level arrays are
    // the parts' blocks (a 2x2 placeholder level is created and dropped)
    mgx_ctx *c = nullptr;
    CHK(create_ctx(&c, 2, 1, dt, nu, &o, nullptr));
    for (auto &L : c->lv) {
        (void)hipFree(L.u[0]);
        (void)hipFree(L.u[1]);
        (void)hipFree(L.rhs);
        (void)hipFree(L.v1);
        (void)hipFree(L.v2);
    }
    c->lv.clear();
    c->N = n;
    c->L = maxlvl;
    c->dist = new Dist();
    *cp = c;
    (void)out;
    return MGX_OK;
}

}  // namespace mgxi

using namespace mgxi;

extern "C" {

int mgx_partition(long n, int maxlvl, int world, int rank, int level, int *ra, int *rb,
                  int *replicated_level) {
    if (n < 2 || maxlvl < 1 || world < 1 || rank < 0 || rank >= world || level < 0 ||
        level >= maxlvl)
        return fail(MGX_E_ARG, "mgx_partition: bad args");
    const int la = plan_la(n, maxlvl, world);
    if (replicated_level) *replicated_level = la;
    if (level >= la) {   // replicated: every rank holds all rows
        if (ra) *ra = 0;
        if (rb) *rb = (int)(n >> level) + 1;
    } else {
        int a, b;
        plan_rows(n, level, world, rank, &a, &b);
        if (ra) *ra = a;
        if (rb) *rb = b;
    }
    return MGX_OK;
}

int mgx_exchange_plan(long n, int maxlvl, int world, int rank, int level, int *count,
                      int *xfers, int cap) {
    if (n < 2 || (n & (n - 1)) || maxlvl < 1 || world < 1 || (world & (world - 1)) ||
        rank < 0 || rank >= world || level < 0 || level >= maxlvl || !count)
        return fail(MGX_E_ARG, "mgx_exchange_plan: bad args");
    std::vector<Xfer> plan;
    if (level < plan_la(n, maxlvl, world)) ghost_plan(n, level, world, rank, plan);
    *count = (int)plan.size();
    if ((int)plan.size() > cap || (!xfers && !plan.empty()))
        return fail(MGX_E_ARG, "mgx_exchange_plan: output too small");
    for (size_t i = 0; i < plan.size(); ++i) {
        int *o = xfers + 5 * i;
        o[0] = plan[i].peer;
        o[1] = plan[i].send_row;
        o[2] = plan[i].send_rows;
        o[3] = plan[i].recv_row;
        o[4] = plan[i].recv_rows;
    }
    return MGX_OK;
}

int mgx_gather_plan(long n, int maxlvl, int world, int rank, int *level, int *row0,
                    int *rows) {
    if (n < 2 || maxlvl < 1 || world < 1 || rank < 0 || rank >= world)
        return fail(MGX_E_ARG, "mgx_gather_plan: bad args");
    const int la = plan_la(n, maxlvl, world);
    long r0, q;
    gather_rows(n, la, world, rank, &r0, &q);
    if (level) *level = la;
    if (row0) *row0 = (int)r0;
    if (rows) *rows = (int)q;
    return MGX_OK;
}

int mgx_dist_unique_id(void *id128) {
    if (!id128) return fail(MGX_E_ARG, "null id");
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    memcpy(id128, &id, sizeof(id));
    return MGX_OK;
}

static int check_world(long n, int maxlvl, int world) {
    if (world < 1 || (world & (world - 1)))
        return fail(MGX_E_ARG, "world size must be a power of two");
    if (maxlvl < 1 || (n >> (maxlvl - 1)) < 2) return fail(MGX_E_ARG, "bad maxlvl");
    if (world > 1 && n / world < 2 * kGhost) return fail(MGX_E_ARG, "too many ranks for n");
    return MGX_OK;
}

int mgx_create_dist(mgx_ctx **out, long n, int maxlvl, double dt, double nu,
                    const mgx_options *opt, int rank, int world, const void *id128) {
    if (!out || !id128 || rank < 0 || rank >= world) return fail(MGX_E_ARG, "mgx_create_dist: bad args");
    *out = nullptr;
    CHK(check_world(n, maxlvl, world));
    if (n < 2 || (n & (n - 1))) return fail(MGX_E_ARG, "n must be a power of two");
    mgx_ctx *c = nullptr;
    CHK(create_dist_common(out, n, maxlvl, dt, nu, opt, &c));
    c->dist->local = false;
    {   // also for world == 1, so the download/norm collectives take one path
        ncclUniqueId id;
        memcpy(&id, id128, sizeof(id));
        ncclResult_t r = ncclCommInitRank(&c->dist->comm, world, id, rank);
        if (r != ncclSuccess) {
            free_ctx(c);
            return fail(MGX_E_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        }
        // (one communicator: the side stream's exchanges use it too, chained
        // after the compute stream's operations by comm_op -- no split
        // communicator whose creation could fail on some ranks only)
    }
    int rc = build_dist(c, world, {rank});
    if (rc) {
        free_ctx(c);
        return rc;
    }
    *out = c;
    return MGX_OK;
}

int mgx_create_local_dist(mgx_ctx **out, long n, int maxlvl, double dt, double nu,
                          const mgx_options *opt, int world) {
    if (!out) return fail(MGX_E_ARG, "mgx_create_local_dist: null out");
    *out = nullptr;
    CHK(check_world(n, maxlvl, world));
    if (n < 2 || (n & (n - 1))) return fail(MGX_E_ARG, "n must be a power of two");
    mgx_ctx *c = nullptr;
    CHK(create_dist_common(out, n, maxlvl, dt, nu, opt, &c));
    c->dist->local = true;
    std::vector<int> ranks;
    for (int r = 0; r < world; ++r) ranks.push_back(r);
    int rc = build_dist(c, world, ranks);
    if (rc) {
        free_ctx(c);
        return rc;
    }
    *out = c;
    return MGX_OK;
}

int mgx_dist_rows(mgx_ctx *c, int part, int *lo, int *hi) {
    if (!c || !c->dist || part < 0 || part >= (int)c->dist->parts.size() ||
        c->dist->parts[part].lv.empty())
        return fail(MGX_E_ARG, "mgx_dist_rows: not a partitioned context / bad part");
    const PLevel &L = c->dist->parts[part].lv[0];
    if (lo) *lo = L.lo;
    if (hi) *hi = L.hi;
    return MGX_OK;
}

int mgx_upload_rows(mgx_ctx *c, const double *const *u0, const double *const *v1,
                    const double *const *v2) {
    if (!c || !c->dist) return fail(MGX_E_ARG, "mgx_upload_rows: not a partitioned context");
    return dist_upload_rows_impl(c, u0, v1, v2);
}

int mgx_dist_info(mgx_ctx *c, int *world, int *rank, int *replicated_level) {
    if (!c) return fail(MGX_E_ARG, "null ctx");
    Dist *d = c->dist;
    if (world) *world = d ? d->world : 1;
    if (rank) *rank = d ? (d->local ? -1 : d->parts[0].rank) : 0;
    if (replicated_level) *replicated_level = d ? d->la : c->L;
    return MGX_OK;
}

}  // extern "C"
