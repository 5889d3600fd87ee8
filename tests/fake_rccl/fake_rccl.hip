// fake_rccl.hip -- TEST INFRASTRUCTURE ONLY (never linked into libmgx.so).
//
// An in-process stand-in for exactly the RCCL entry points dist.hip calls:
// ncclGetUniqueId, ncclCommInitRank / ncclCommSplit / ncclCommDestroy, ncclGroupStart /
// ncclGroupEnd, ncclSend / ncclRecv, ncclAllGather, ncclAllReduce (sum),
// ncclBroadcast, ncclGetErrorString.  Ranks are host THREADS of one process,
// all on one GPU, so libmgx's real RCCL code path (dist.hip, the branch a
// one-process-per-GPU run takes) executes with peers on a one-GPU box, where
// the real RCCL refuses two ranks on one device ("host-thread fake
// transport").
//
// Semantics kept from NCCL (what the test is for):
//   * stream ordering: an operation starts when the ISSUING stream reaches it
//     (an event recorded at the call) and every participating stream waits for
//     its completion (events back) -- a missing fork/join in the caller shows
//     up as a race, not as a silently serialised result;
//   * matching: sends and receives pair up per (sender, receiver) in posting
//     order, byte counts must agree; collectives must be called in the same
//     order with the same type/count/root on every rank;
//   * in-place all-gather (sendbuff == recvbuff + rank*count) and broadcast;
//     any other overlap of send and receive buffers is rejected, as are
//     buffers that run past the end of their device allocation.
//   * one operation at a time per rank: NCCL operations of a communicator must
//     not run concurrently (and those of two communicators may deadlock), so
//     every operation a rank issues must be ORDERED after its previous one on
//     the device -- the same stream, or an event chain.  A happens-before
//     model checks that deterministically, whatever the timing: libmgx's
//     hipEventRecord / hipStreamWaitEvent / hip*Synchronize calls are wrapped
//     (-Wl,--wrap, tests/fake_rccl/Makefile) into vector clocks per stream,
//     event and host thread; an operation on stream s whose clock does not
//     cover the rank's previous operation is counted as a violation
//     (fake_rccl_order_violations).  The fake's own event calls use the real
//     functions, so peers never create the order a rank must create itself.
// Data moves as device-to-device hipMemcpyAsync on the receiver's stream;
// the all-reduce sums the ranks' values in rank order with a small kernel.
// libmgx_fakerccl.so = libmgx's own objects + this file, linked -Bsymbolic
// (tests/fake_rccl/Makefile).  Counters per entry point let the test assert
// that every call site ran.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

// libmgx's calls land in the __wrap_ functions below; the fake's own go
// straight to the HIP runtime
extern "C" {
hipError_t __real_hipEventRecord(hipEvent_t e, hipStream_t s);
hipError_t __real_hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned int flags);
hipError_t __real_hipStreamSynchronize(hipStream_t s);
hipError_t __real_hipEventSynchronize(hipEvent_t e);
hipError_t __real_hipDeviceSynchronize(void);
}

namespace fk {

enum Fn { kInit, kDestroy, kGroupStart, kGroupEnd, kSend, kRecv, kAllGather, kAllReduce,
          kBroadcast, kUniqueId, kSplit, kNumFn };
const char *kFnNames[kNumFn] = {"ncclCommInitRank", "ncclCommDestroy", "ncclGroupStart",
                                "ncclGroupEnd", "ncclSend", "ncclRecv", "ncclAllGather",
                                "ncclAllReduce", "ncclBroadcast", "ncclGetUniqueId",
                                "ncclCommSplit"};
std::atomic<long> g_calls[kNumFn];
thread_local long t_calls[kNumFn];   // the calling thread's (one rank's) calls
std::atomic<long> g_bytes{0};
std::mutex g_err_mu;
std::string g_err;   // first failure, process-wide (read by the test)

ncclResult_t bad(ncclResult_t r, const std::string &msg) {
    std::lock_guard<std::mutex> g(g_err_mu);
    if (g_err.empty()) g_err = msg;
    fprintf(stderr, "fake_rccl: %s\n", msg.c_str());
    return r;
}

// ---- happens-before model (vector clocks) of the issuing threads' streams
namespace hb {
using VC = std::map<hipStream_t, long>;   // stream -> operations of it covered
void join(VC &a, const VC &b) {
    for (const auto &kv : b) {
        long &x = a[kv.first];
        if (kv.second > x) x = kv.second;
    }
}
std::mutex mu;
std::map<hipStream_t, VC> streams;   // what the work enqueued on a stream so far follows
std::map<hipEvent_t, VC> events;     // the clock its last record captured
thread_local VC host;                // what this host thread has synchronised with
struct Last {
    bool any = false;
    hipStream_t st = nullptr;
    long tick = 0;
    std::string what;
};
thread_local Last last;   // this thread's (rank's) previous RCCL operation
std::atomic<long> violations{0};
std::string first;        // the first violation (under mu)

// an RCCL operation of the calling rank issued on st
void op(hipStream_t st, const char *what) {
    std::lock_guard<std::mutex> g(mu);
    VC &v = streams[st];
    join(v, host);
    if (last.any && last.st != st) {
        const auto it = v.find(last.st);
        const long seen = it == v.end() ? 0 : it->second;
        if (seen < last.tick) {
            if (violations++ == 0)
                first = std::string(what) + " on stream " + std::to_string((uintptr_t)st) +
                        " is not ordered after the rank's previous operation (" + last.what +
                        " on stream " + std::to_string((uintptr_t)last.st) + ")";
        }
    }
    const long t = ++v[st];
    last = Last{true, st, t, what};
}
}  // namespace hb

size_t type_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

// [p, p+bytes) must lie inside one device allocation
bool in_allocation(const void *p, size_t bytes) {
    if (bytes == 0) return true;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, const_cast<void *>(p)) != hipSuccess) return false;
    const char *b = static_cast<const char *>(base), *q = static_cast<const char *>(p);
    return q >= b && q + bytes <= b + size;
}

struct P2P {
    const void *src = nullptr;
    size_t bytes = 0;
    hipEvent_t ready = nullptr;   // the sender's stream reached the send
    hipEvent_t done = nullptr;    // the receiver's copy has finished
    bool matched = false;
    bool failed = false;
};

enum CollKind { kCollAllGather, kCollAllReduce, kCollBroadcast };

struct Coll {
    CollKind kind;
    size_t count;
    ncclDataType_t type;
    int root;
    std::vector<const void *> send;
    std::vector<void *> recv;
    std::vector<hipEvent_t> ready, read_done;
    int nready = 0, nread = 0, nleft = 0;
    bool mismatch = false;
};

struct Clique {
    int world = 0, joined = 0, alive = 0;
    std::vector<bool> ranks;
    std::mutex mu;
    std::condition_variable cv;
    std::map<std::pair<int, int>, std::deque<std::shared_ptr<P2P>>> mail;   // (src, dst)
    std::map<long, std::shared_ptr<Coll>> colls;
};

std::mutex g_mu;
std::map<std::string, std::shared_ptr<Clique>> g_cliques;

struct Op {
    bool send;
    ncclComm_t comm;
    void *buf;
    size_t bytes;
    int peer;
    hipStream_t st;
};
thread_local int t_depth = 0;
thread_local std::vector<Op> t_ops;

}  // namespace fk

struct ncclComm {
    std::shared_ptr<fk::Clique> q;
    std::string key;
    int rank = 0, world = 0;
    long seq = 0;                      // collectives issued by this rank
    long splits = 0;                   // ncclCommSplit calls by this rank
    std::vector<hipEvent_t> events;    // destroyed with the communicator
    double *stage = nullptr;           // all-reduce staging (this rank's stream only)
    size_t stage_bytes = 0;
    hipEvent_t event() {
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
        events.push_back(e);
        return e;
    }
};

namespace fk {

__global__ void k_sum_ranks(double *out, const double *stage, size_t count, int world) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    double s = stage[i];
    for (int r = 1; r < world; ++r) s = s + stage[(size_t)r * count + i];
    out[i] = s;
}

// Execute this thread's queued point-to-point operations (one group).
ncclResult_t flush_group() {
    std::vector<Op> ops;
    ops.swap(t_ops);
    if (ops.empty()) return ncclSuccess;
    ncclResult_t rc = ncclSuccess;
    // 1. every stream with an operation: where it stands now
    std::map<hipStream_t, hipEvent_t> ready;
    for (const Op &o : ops) {
        if (ready.count(o.st)) continue;
        hb::op(o.st, "a send/recv group");
        hipEvent_t e = o.comm->event();
        if (!e || __real_hipEventRecord(e, o.st) != hipSuccess)
            return bad(ncclUnhandledCudaError, "event record");
        ready[o.st] = e;
    }
    // 2. post the sends
    std::vector<std::pair<const Op *, std::shared_ptr<P2P>>> posted;
    for (const Op &o : ops) {
        if (!o.send) continue;
        auto p = std::make_shared<P2P>();
        p->src = o.buf;
        p->bytes = o.bytes;
        p->ready = ready[o.st];
        Clique &q = *o.comm->q;
        {
            std::lock_guard<std::mutex> g(q.mu);
            q.mail[{o.comm->rank, o.peer}].push_back(p);
        }
        q.cv.notify_all();
        posted.push_back({&o, p});
    }
    // 3. match the receives in order, copy on the receiving stream
    std::map<hipStream_t, std::vector<std::pair<Clique *, std::shared_ptr<P2P>>>> got;
    for (const Op &o : ops) {
        if (o.send) continue;
        Clique &q = *o.comm->q;
        std::shared_ptr<P2P> p;
        {
            std::unique_lock<std::mutex> g(q.mu);
            auto &box = q.mail[{o.peer, o.comm->rank}];
            q.cv.wait(g, [&] { return !box.empty(); });
            p = box.front();
            box.pop_front();
        }
        if (p->bytes != o.bytes) {
            p->failed = true;
            rc = bad(ncclInvalidUsage, "recv of " + std::to_string(o.bytes) + " B from rank " +
                                           std::to_string(o.peer) + " matched a send of " +
                                           std::to_string(p->bytes) + " B");
        } else if (__real_hipStreamWaitEvent(o.st, p->ready, 0) != hipSuccess ||
                   hipMemcpyAsync(o.buf, p->src, o.bytes, hipMemcpyDeviceToDevice, o.st) !=
                       hipSuccess) {
            rc = bad(ncclUnhandledCudaError, "p2p copy");
        }
        g_bytes += (long)o.bytes;
        got[o.st].push_back({o.comm->q.get(), p});
    }
    // 4. hand the completion back to the senders
    for (auto &kv : got) {
        hipEvent_t done = ops[0].comm->event();
        if (!done || __real_hipEventRecord(done, kv.first) != hipSuccess)
            rc = bad(ncclUnhandledCudaError, "event record");
        for (auto &qp : kv.second) {
            std::lock_guard<std::mutex> g(qp.first->mu);
            qp.second->done = done;
            qp.second->matched = true;
        }
    }
    for (const Op &o : ops) o.comm->q->cv.notify_all();
    // 5. the sending streams wait until their data has been taken
    for (auto &sp : posted) {
        Clique &q = *sp.first->comm->q;
        {
            std::unique_lock<std::mutex> g(q.mu);
            q.cv.wait(g, [&] { return sp.second->matched; });
        }
        if (sp.second->failed)
            rc = bad(ncclInvalidUsage, "send of " + std::to_string(sp.second->bytes) +
                                           " B to rank " + std::to_string(sp.first->peer) +
                                           " did not match its receive");
        if (sp.second->done && __real_hipStreamWaitEvent(sp.first->st, sp.second->done, 0) != hipSuccess)
            rc = bad(ncclUnhandledCudaError, "stream wait");
    }
    return rc;
}

ncclResult_t enqueue(bool send, void *buf, size_t count, ncclDataType_t t, int peer,
                     ncclComm_t comm, hipStream_t st) {
    if (!comm) return bad(ncclInvalidArgument, "null communicator");
    const size_t es = type_size(t);
    if (!es) return bad(ncclInvalidArgument, "unsupported data type");
    if (peer < 0 || peer >= comm->world || peer == comm->rank)
        return bad(ncclInvalidArgument, "bad peer " + std::to_string(peer));
    if (!buf || !in_allocation(buf, count * es))
        return bad(ncclInvalidArgument, std::string(send ? "send" : "recv") +
                                            " buffer outside its device allocation");
    t_ops.push_back({send, comm, buf, count * es, peer, st});
    if (t_depth == 0) return flush_group();   // an operation outside a group
    return ncclSuccess;
}

// A collective: (1) every rank publishes its buffers and where its stream
// stands, (2) reads what it needs from the others on its own stream,
// (3) waits until every rank has read (in-place buffers), (4) reduces.
ncclResult_t collective(CollKind kind, const void *send, void *recv, size_t count,
                        ncclDataType_t t, int root, ncclComm_t comm, hipStream_t st) {
    if (!comm) return bad(ncclInvalidArgument, "null communicator");
    if (t_depth > 0) return bad(ncclInvalidUsage, "collective inside a group (unsupported)");
    const size_t es = type_size(t);
    if (!es) return bad(ncclInvalidArgument, "unsupported data type");
    const int R = comm->world, me = comm->rank;
    const size_t bytes = count * es;
    const size_t rbytes = kind == kCollAllGather ? bytes * R : bytes;
    if (!in_allocation(recv, rbytes) || !in_allocation(send, bytes))
        return bad(ncclInvalidArgument, "collective buffer outside its device allocation");
    if (kind == kCollAllGather && send != recv) {
        const char *s = static_cast<const char *>(send), *r = static_cast<const char *>(recv);
        const bool in_place = s == r + (size_t)me * bytes;
        if (!in_place && s < r + rbytes && r < s + bytes)
            return bad(ncclInvalidArgument, "all-gather buffers overlap but are not in place");
    }
    if (kind == kCollAllReduce && (t != ncclFloat64))
        return bad(ncclInvalidArgument, "all-reduce: only double sums are implemented");
    Clique &q = *comm->q;
    hb::op(st, kind == kCollAllGather ? "an all-gather" : kind == kCollAllReduce ? "an all-reduce"
                                                                                : "a broadcast");
    hipEvent_t ready = comm->event();
    if (!ready || __real_hipEventRecord(ready, st) != hipSuccess)
        return bad(ncclUnhandledCudaError, "event record");
    const long seq = comm->seq++;
    std::shared_ptr<Coll> c;
    {
        std::unique_lock<std::mutex> g(q.mu);
        auto &slot = q.colls[seq];
        if (!slot) {
            slot = std::make_shared<Coll>();
            slot->kind = kind;
            slot->count = count;
            slot->type = t;
            slot->root = root;
            slot->send.assign(R, nullptr);
            slot->recv.assign(R, nullptr);
            slot->ready.assign(R, nullptr);
            slot->read_done.assign(R, nullptr);
        }
        c = slot;
        if (c->kind != kind || c->count != count || c->type != t || c->root != root)
            c->mismatch = true;
        c->send[me] = send;
        c->recv[me] = recv;
        c->ready[me] = ready;
        c->nready++;
        q.cv.notify_all();
        q.cv.wait(g, [&] { return c->nready == R; });
    }
    ncclResult_t rc = ncclSuccess;
    if (c->mismatch) rc = bad(ncclInvalidUsage, "collective #" + std::to_string(seq) +
                                                    " differs between ranks");
    // (2) reads on my stream
    double *stage = nullptr;
    auto cp = [&](void *dst, const void *src, size_t n, int from) {
        if (__real_hipStreamWaitEvent(st, c->ready[from], 0) != hipSuccess ||
            hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, st) != hipSuccess)
            rc = bad(ncclUnhandledCudaError, "collective copy");
        g_bytes += (long)n;
    };
    if (rc == ncclSuccess) {
        if (kind == kCollAllGather) {
            for (int r = 0; r < R; ++r) {
                char *dst = static_cast<char *>(recv) + (size_t)r * bytes;
                if (r == me) {
                    if (send != dst) cp(dst, send, bytes, me);
                } else {
                    cp(dst, c->send[r], bytes, r);
                }
            }
        } else if (kind == kCollBroadcast) {
            if (me != root || send != recv) cp(recv, c->send[root], bytes, root);
        } else {
            // a persistent per-rank staging buffer, used in this rank's stream
            // order only (grown, with a device sync, for a larger count)
            if (comm->stage_bytes < bytes * R) {
                (void)__real_hipDeviceSynchronize();
                (void)hipFree(comm->stage);
                comm->stage = nullptr;
                comm->stage_bytes = 0;
                if (hipMalloc((void **)&comm->stage, bytes * R) == hipSuccess)
                    comm->stage_bytes = bytes * R;
                else
                    rc = bad(ncclUnhandledCudaError, "staging alloc");
            }
            stage = comm->stage;
            for (int r = 0; rc == ncclSuccess && r < R; ++r)
                cp(reinterpret_cast<char *>(stage) + (size_t)r * bytes, c->send[r], bytes, r);
        }
    }
    hipEvent_t rd = comm->event();
    if (!rd || __real_hipEventRecord(rd, st) != hipSuccess) rc = bad(ncclUnhandledCudaError, "event");
    {   // (3)
        std::unique_lock<std::mutex> g(q.mu);
        c->read_done[me] = rd;
        c->nread++;
        q.cv.notify_all();
        q.cv.wait(g, [&] { return c->nread == R; });
    }
    for (int r = 0; r < R; ++r)
        if (r != me && __real_hipStreamWaitEvent(st, c->read_done[r], 0) != hipSuccess)
            rc = bad(ncclUnhandledCudaError, "stream wait");
    // (4)
    if (kind == kCollAllReduce && stage && rc == ncclSuccess) {
        const unsigned blocks = (unsigned)((count + 255) / 256);
        hipLaunchKernelGGL(k_sum_ranks, dim3(blocks ? blocks : 1), dim3(256), 0, st,
                           static_cast<double *>(recv), stage, count, R);
        if (hipGetLastError() != hipSuccess) rc = bad(ncclUnhandledCudaError, "sum kernel");
    }
    {
        std::lock_guard<std::mutex> g(q.mu);
        if (++c->nleft == R) q.colls.erase(seq);
    }
    return rc;
}

}  // namespace fk

using namespace fk;

extern "C" {

const char *ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (fake rccl)";
        case ncclUnhandledCudaError: return "HIP call failed (fake rccl)";
        case ncclInvalidArgument: return "invalid argument (fake rccl)";
        case ncclInvalidUsage: return "invalid usage (fake rccl)";
        default: return "error (fake rccl)";
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
    static std::atomic<long> ctr{0};
    g_calls[kUniqueId]++;
    t_calls[kUniqueId]++;
    if (!id) return bad(ncclInvalidArgument, "null id");
    memset(id, 0, sizeof(*id));
    snprintf(id->internal, sizeof(id->internal), "fake-rccl:%d:%ld", (int)getpid(), ctr++);
    return ncclSuccess;
}

static ncclResult_t init_rank(ncclComm_t *out, int nranks, const std::string &key, int rank) {
    std::shared_ptr<Clique> q;
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto &slot = g_cliques[key];
        if (!slot) {
            slot = std::make_shared<Clique>();
            slot->world = nranks;
            slot->ranks.assign(nranks, false);
        }
        q = slot;
    }
    std::unique_lock<std::mutex> g(q->mu);
    if (q->world != nranks || q->ranks[rank])
        return bad(ncclInvalidUsage, "ncclCommInitRank: world mismatch or rank joined twice");
    q->ranks[rank] = true;
    q->joined++;
    q->alive++;
    q->cv.notify_all();
    q->cv.wait(g, [&] { return q->joined == q->world; });   // init is collective
    g.unlock();
    ncclComm_t c = new ncclComm();
    c->q = q;
    c->key = key;
    c->rank = rank;
    c->world = nranks;
    if (hipMalloc((void **)&c->stage, 1 << 16) != hipSuccess)
        return bad(ncclUnhandledCudaError, "staging alloc");
    c->stage_bytes = 1 << 16;
    {   // load the sum kernel once, outside any concurrent launch
        static std::mutex warm_mu;
        static bool warm = false;
        std::lock_guard<std::mutex> w(warm_mu);
        if (!warm) {
            hipLaunchKernelGGL(k_sum_ranks, dim3(1), dim3(256), 0, nullptr, c->stage, c->stage,
                               (size_t)0, 1);
            if (__real_hipDeviceSynchronize() != hipSuccess)
                return bad(ncclUnhandledCudaError, "sum kernel warm-up");
            warm = true;
        }
    }
    *out = c;
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *out, int nranks, ncclUniqueId id, int rank) {
    g_calls[kInit]++;
    t_calls[kInit]++;
    if (!out || nranks < 1 || rank < 0 || rank >= nranks)
        return bad(ncclInvalidArgument, "ncclCommInitRank: bad args");
    return init_rank(out, nranks, std::string(id.internal, sizeof(id.internal)), rank);
}

// Only the split libmgx makes: every rank the same colour, key = its rank, so
// the new communicator has the parent's ranks (a fresh clique: its own
// mailboxes and collective sequence, as a separate NCCL communicator has).
// The k-th split of a parent on every rank joins the same clique.
ncclResult_t ncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t *out,
                           ncclConfig_t *config) {
    g_calls[kSplit]++;
    t_calls[kSplit]++;
    (void)config;
    if (!comm || !out) return bad(ncclInvalidArgument, "ncclCommSplit: bad args");
    if (color != 0 || key != comm->rank)
        return bad(ncclInvalidArgument, "ncclCommSplit: only colour 0 with key = rank is faked");
    const std::string k = comm->key + "/split" + std::to_string(comm->splits++);
    return init_rank(out, comm->world, k, comm->rank);
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
    g_calls[kDestroy]++;
    t_calls[kDestroy]++;
    if (!c) return ncclSuccess;
    for (hipEvent_t e : c->events) {
        (void)__real_hipEventSynchronize(e);
        (void)hipEventDestroy(e);
    }
    (void)hipFree(c->stage);
    bool last;
    {
        std::lock_guard<std::mutex> g(c->q->mu);
        last = --c->q->alive == 0;
    }
    if (last) {
        std::lock_guard<std::mutex> g(g_mu);
        g_cliques.erase(c->key);
    }
    delete c;
    return ncclSuccess;
}

ncclResult_t ncclGroupStart(void) {
    g_calls[kGroupStart]++;
    t_calls[kGroupStart]++;
    ++t_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd(void) {
    g_calls[kGroupEnd]++;
    t_calls[kGroupEnd]++;
    if (t_depth <= 0) return bad(ncclInvalidUsage, "ncclGroupEnd without ncclGroupStart");
    if (--t_depth > 0) return ncclSuccess;
    return flush_group();
}

ncclResult_t ncclSend(const void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm,
                      hipStream_t st) {
    g_calls[kSend]++;
    t_calls[kSend]++;
    return enqueue(true, const_cast<void *>(buf), count, t, peer, comm, st);
}

ncclResult_t ncclRecv(void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm,
                      hipStream_t st) {
    g_calls[kRecv]++;
    t_calls[kRecv]++;
    return enqueue(false, buf, count, t, peer, comm, st);
}

ncclResult_t ncclAllGather(const void *send, void *recv, size_t count, ncclDataType_t t,
                           ncclComm_t comm, hipStream_t st) {
    g_calls[kAllGather]++;
    t_calls[kAllGather]++;
    return collective(kCollAllGather, send, recv, count, t, 0, comm, st);
}

ncclResult_t ncclAllReduce(const void *send, void *recv, size_t count, ncclDataType_t t,
                           ncclRedOp_t op, ncclComm_t comm, hipStream_t st) {
    g_calls[kAllReduce]++;
    t_calls[kAllReduce]++;
    if (op != ncclSum) return bad(ncclInvalidArgument, "all-reduce: only ncclSum is implemented");
    return collective(kCollAllReduce, send, recv, count, t, 0, comm, st);
}

ncclResult_t ncclBroadcast(const void *send, void *recv, size_t count, ncclDataType_t t,
                           int root, ncclComm_t comm, hipStream_t st) {
    g_calls[kBroadcast]++;
    t_calls[kBroadcast]++;
    if (!comm || root < 0 || root >= comm->world)
        return bad(ncclInvalidArgument, "broadcast: bad root");
    return collective(kCollBroadcast, send, recv, count, t, root, comm, st);
}

// ---- libmgx's stream-order calls (-Wl,--wrap): the happens-before model
hipError_t __wrap_hipEventRecord(hipEvent_t e, hipStream_t s) {
    {
        std::lock_guard<std::mutex> g(hb::mu);
        hb::VC &v = hb::streams[s];
        hb::join(v, hb::host);
        hb::events[e] = v;
    }
    return __real_hipEventRecord(e, s);
}
hipError_t __wrap_hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned int flags) {
    {
        std::lock_guard<std::mutex> g(hb::mu);
        hb::VC &v = hb::streams[s];
        hb::join(v, hb::host);
        const auto it = hb::events.find(e);
        if (it != hb::events.end()) hb::join(v, it->second);
    }
    return __real_hipStreamWaitEvent(s, e, flags);
}
hipError_t __wrap_hipStreamSynchronize(hipStream_t s) {
    const hipError_t r = __real_hipStreamSynchronize(s);
    std::lock_guard<std::mutex> g(hb::mu);
    hb::join(hb::host, hb::streams[s]);
    return r;
}
hipError_t __wrap_hipEventSynchronize(hipEvent_t e) {
    const hipError_t r = __real_hipEventSynchronize(e);
    std::lock_guard<std::mutex> g(hb::mu);
    const auto it = hb::events.find(e);
    if (it != hb::events.end()) hb::join(hb::host, it->second);
    return r;
}
hipError_t __wrap_hipDeviceSynchronize(void) {
    const hipError_t r = __real_hipDeviceSynchronize();
    std::lock_guard<std::mutex> g(hb::mu);
    for (const auto &kv : hb::streams) hb::join(hb::host, kv.second);
    return r;
}

// ---- test hooks
// 1 if the calling thread (rank) has synchronised on the host with the end of
// its last RCCL operation (none is in flight from its point of view)
int fake_rccl_rank_idle(void) {
    std::lock_guard<std::mutex> g(hb::mu);
    if (!hb::last.any) return 1;
    const auto it = hb::host.find(hb::last.st);
    return it != hb::host.end() && it->second >= hb::last.tick ? 1 : 0;
}
// RCCL operations (of any rank) issued while the rank's previous one was not
// ordered before them, and the first such case
long fake_rccl_order_violations(void) { return hb::violations.load(); }
const char *fake_rccl_order_message(void) {
    static thread_local std::string m;
    std::lock_guard<std::mutex> g(hb::mu);
    m = hb::first;
    return m.c_str();
}
long fake_rccl_calls(const char *name) {
    for (int i = 0; i < kNumFn; ++i)
        if (!strcmp(name, kFnNames[i])) return g_calls[i].load();
    return -1;
}
long fake_rccl_bytes(void) { return g_bytes.load(); }
// the calls made by the calling thread (one rank) so far
long fake_rccl_thread_calls(const char *name) {
    for (int i = 0; i < kNumFn; ++i)
        if (!strcmp(name, kFnNames[i])) return t_calls[i];
    return -1;
}
const char *fake_rccl_error(void) {
    std::lock_guard<std::mutex> g(g_err_mu);
    return g_err.c_str();
}
void fake_rccl_reset(void) {
    for (auto &c : g_calls) c = 0;
    g_bytes = 0;
    hb::violations = 0;
    {
        std::lock_guard<std::mutex> g(hb::mu);
        hb::first.clear();
    }
    std::lock_guard<std::mutex> g(g_err_mu);
    g_err.clear();
}

}  // extern "C"
