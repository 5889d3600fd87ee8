// plan.h -- the multi-GPU row partition and its exchange plan.
//
// Host-only C++ (no HIP, no RCCL): dist.hip executes these plans over RCCL or
// over device copies, and tests/asan/plan_asan.cpp builds this header alone
// with AddressSanitizer / UBSan to check every plan on the CPU.
//
// Levels 0..la-1 are split into contiguous row blocks, one per rank, with
// boundaries at even rows (restriction rows 2I and prolongation parents stay
// local); each block also holds kGhost = 16 ghost rows of its neighbours on
// every level: the cross-cycle pass's cone on level 0 is 14 rows, and on the
// coarser levels a post-smoothing pass computes kPostExt rows past its block
// as well (communication-avoiding: the finer level's prolongation then needs
// no exchange of the corrected u), a cone of kPostExt + 2K <= 16 rows.
#pragma once
#include <algorithm>
#include <string>
#include <vector>

namespace mgxplan {

constexpr int kGhost = 16;       // >= the widest cone (see above)
constexpr int kGhostFine = 16;   // level 0: the cross-cycle pass's cone is 14 rows
// Rows past its block (each side) a coarse level's post-smoothing pass
// computes: the finer level's pass with a cone of c rows (its output + its
// stages) reads coarse rows ra/2 - c/2 .. rb/2 + c/2 (the odd row's second
// parent): c = 14 for the cross pass, kPostExt + 2K <= 16 for a coarse post
// pass, so 10 rows (even: row blocks start at even rows) cover every level.
constexpr int kPostExt = 10;

// Rows [ra, rb) of level l owned by `rank` (the same rule on every rank; the
// last rank also owns the boundary row n).
inline void plan_rows(long n0, int l, int world, int rank, int *ra, int *rb) {
    const long nl = n0 >> l;
    const long q = nl / world;
    *ra = (int)(rank * q);
    *rb = rank == world - 1 ? (int)nl + 1 : (int)((rank + 1) * q);
}

// First replicated level: the first whose blocks would be shorter than
// min_rows (at most L-1: the coarsest level is always replicated).
inline int plan_la(long n0, int L, int world, long min_rows) {
    if (world <= 1) return L - 1 > 0 ? L - 1 : 0;
    int la = 0;
    while (la < L - 1 && ((n0 >> la) / world) >= min_rows) ++la;
    return la;
}

inline int ghost_width(int l) { return l == 0 ? kGhostFine : kGhost; }

// Allocated rows [lo, hi] of `rank` on level l: owned + ghosts, clipped.
inline void alloc_rows(long n0, int l, int world, int rank, int *ra, int *rb, int *lo,
                       int *hi) {
    plan_rows(n0, l, world, rank, ra, rb);
    const int g = ghost_width(l);
    *lo = std::max(0, *ra - g);
    *hi = (int)std::min<long>(n0 >> l, (long)*rb - 1 + g);
}

// The all-gather into the first replicated level la: rank r contributes rows
// [r*q, (r+1)*q), q = n_la / world (what its restriction from its level la-1
// block writes; row n_la, the boundary, is never read), in place, rank-major.
inline void gather_rows(long n0, int la, int world, int rank, long *row0, long *rows) {
    const long q = (n0 >> la) / world;
    *row0 = rank * q;
    *rows = q;
}

// ---- exchange plan.  ONE host-side description of every ghost-row transfer,
// consumed by both transports of dist.hip: RCCL posts each entry as an
// ncclSend of its send rows + an ncclRecv into its recv rows; the local
// (virtual-rank) transport copies the sender's rows into the peer's rows.  So
// the single-GPU parity tests execute exactly the offsets / counts the RCCL
// ranks post.  Rows are global row indices of the level.
struct Xfer {
    int peer;
    int send_row, send_rows;   // send rows [send_row, +send_rows) to peer
    int recv_row, recv_rows;   // receive rows [recv_row, +recv_rows) from it
};

// Ghost rows of level l of `rank`: [lo, ra) come from rank-1 (its last owned
// rows), [rb, hi] from rank+1 (its first owned rows); it sends each
// neighbour the rows that neighbour's ghosts mirror.
inline void ghost_plan(long n0, int l, int world, int rank, std::vector<Xfer> &out) {
    out.clear();
    if (world <= 1) return;
    int ra, rb, lo, hi;
    alloc_rows(n0, l, world, rank, &ra, &rb, &lo, &hi);
    for (int peer : {rank - 1, rank + 1}) {
        if (peer < 0 || peer >= world) continue;
        int pa, pb, plo, phi;
        alloc_rows(n0, l, world, peer, &pa, &pb, &plo, &phi);
        Xfer x;
        x.peer = peer;
        if (peer < rank) {   // its upper ghosts [pb, phi] = my first owned rows
            x.send_row = pb;
            x.send_rows = phi - pb + 1;
            x.recv_row = lo;
            x.recv_rows = ra - lo;
        } else {             // its lower ghosts [plo, pa) = my last owned rows
            x.send_row = plo;
            x.send_rows = pa - plo;
            x.recv_row = rb;
            x.recv_rows = hi - rb + 1;
        }
        out.push_back(x);
    }
}

// The plans of all ranks agree pairwise (what i sends j is what j receives
// from i: same global rows, same count), sends read only owned rows, receives
// land only in allocated ghost rows.  "" when consistent, else the reason.
inline std::string plan_check(long n0, int l, int world) {
    std::vector<std::vector<Xfer>> P(world);
    for (int r = 0; r < world; ++r) ghost_plan(n0, l, world, r, P[r]);
    for (int r = 0; r < world; ++r) {
        int ra, rb, lo, hi;
        alloc_rows(n0, l, world, r, &ra, &rb, &lo, &hi);
        for (const Xfer &x : P[r]) {
            if (x.send_rows <= 0 || x.send_row < ra || x.send_row + x.send_rows > rb)
                return "exchange plan: send outside the owned rows";
            if (x.recv_rows <= 0 || x.recv_row < lo || x.recv_row + x.recv_rows > hi + 1 ||
                (x.recv_row < rb && x.recv_row + x.recv_rows > ra))
                return "exchange plan: receive outside the ghost rows";
            const Xfer *y = nullptr;
            for (const Xfer &z : P[x.peer])
                if (z.peer == r) y = &z;
            if (!y || y->recv_row != x.send_row || y->recv_rows != x.send_rows)
                return "exchange plan: peers disagree";
        }
    }
    return "";
}

}  // namespace mgxplan
