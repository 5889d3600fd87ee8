// sepvel.h -- exact rank-1 (separable) velocity fields, host only.
//
// The reference's velocity field is an outer product in floating point:
// multigrid.cpp:221-222 evaluates v1 = -ky*sin(kx*i*dx)*cos(ky*j*dx) left to
// right, i.e. v1[i][j] = fl(a_i * b_j) with a_i = fl(-ky*sin(..i..)) and
// b_j = cos(..j..); v2 likewise.  A level pass then needs, per row, two
// numbers instead of two 2-D rows: the smoothers read rhs and u from HBM and
// form t = v*h/2 as fl(a_R * fl(b_c*h/2)) -- bitwise the t of the stored
// field (below) -- which takes 2 of the 5 input streams of the finest level
// off HBM.
//
// factor_rank1 recovers such factors from a stored field EXACTLY or reports
// that there are none: it takes a candidate column j* whose entries are the
// row factors (b_{j*} = 1: cos(0) for v1, sin(pi/2) for v2), picks each
// column factor among the few doubles next to v[p][j] / a_p that reproduce
// the column on several pivot rows p, and then checks EVERY entry bitwise:
// fl(a_i * b_j) == v[i][j] (same bits, signed zeros included).  It also
// requires every nonzero |v| and |b| to stay normal after the h/2 scalings
// the levels use (h/2 >= hmin), so that fl(fl(a*b)*s) == fl(a*fl(b*s)) for
// those powers of two s.  Anything else -- a random field, a rank-2 flow --
// returns false and the solver keeps the 2-D arrays.  Used by mgx.hip at
// upload; exported for tests as mgx_factor_velocity.
#pragma once
#include <algorithm>
#include <atomic>
#include <memory>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace mgxsep {

inline uint64_t bits(double x) {
    uint64_t b;
    std::memcpy(&b, &x, sizeof b);
    return b;
}

template <class F>
inline void parallel_rows(long rows, int nthreads, F &&f) {
    int nt = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
    nt = (int)std::max<long>(1, std::min<long>({(long)nt, 64L, rows}));
    if (nt == 1) {
        f(0L, rows);
        return;
    }
    std::vector<std::thread> th;
    const long per = (rows + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const long a = t * per, b = std::min(rows, a + per);
        if (a < b) th.emplace_back([&f, a, b] { f(a, b); });
    }
    for (auto &x : th) x.join();
}

// v: rows x w, row-major (row stride ld).  On success a[rows], b[w] hold
// exact factors.  smin: the smallest scaling (h/2 of the coarsest level that
// uses the factors); 0 skips the range check.
// jsel (optional): the column j* whose entries ARE the row factors (b_{j*} = 1).
inline bool factor_rank1(const double *v, long rows, long w, long ld, double smin, double *a,
                         double *b, int nthreads = 0, long *jsel = nullptr) {
    if (rows < 1 || w < 1) return false;
    const long cands[5] = {0, w / 2, w - 1, w / 4, (3 * w) / 4};
    constexpr int kC = 9;   // column-factor candidates: q and 4 neighbours each way
    for (int ci = 0; ci < 5; ++ci) {
        const long js = cands[ci];
        bool dup = false;
        for (int k = 0; k < ci; ++k) dup = dup || cands[k] == js;
        if (dup) continue;
        for (long i = 0; i < rows; ++i) a[i] = v[i * ld + js];
        // pivot rows: the largest |a| and up to 31 more nonzero rows spread out
        std::vector<long> piv;
        long ip = -1;
        for (long i = 0; i < rows; ++i)
            if (a[i] != 0.0 && std::isfinite(a[i]) && (ip < 0 || std::fabs(a[i]) > std::fabs(a[ip])))
                ip = i;
        if (ip < 0) continue;
        piv.push_back(ip);
        for (int k = 1; k < 32; ++k) {
            long i = (rows - 1) * k / 32;
            while (i < rows && !(a[i] != 0.0 && std::isfinite(a[i]))) ++i;
            if (i < rows && std::find(piv.begin(), piv.end(), i) == piv.end()) piv.push_back(i);
        }
        // per column: the candidates that reproduce the pivot rows, in order
        std::vector<double> cand((size_t)w * kC);
        std::vector<int> pick(w, -1);
        auto passes = [&](long j, double c) {
            if (!std::isfinite(c)) return false;
            for (long p : piv)
                if (bits(a[p] * c) != bits(v[p * ld + j])) return false;
            return true;
        };
        auto advance = [&](long j) {   // next candidate of column j passing the pivots
            for (int k = pick[j] + 1; k < kC; ++k)
                if (passes(j, cand[(size_t)j * kC + k])) {
                    pick[j] = k;
                    b[j] = cand[(size_t)j * kC + k];
                    return true;
                }
            return false;
        };
        bool ok = true;
        for (long j = 0; j < w && ok; ++j) {
            double *cj = &cand[(size_t)j * kC];
            const double q = v[ip * ld + j] / a[ip];
            cj[0] = q;
            double up = q, dn = q;
            for (int k = 0; k < (kC - 1) / 2; ++k) {
                up = std::nextafter(up, INFINITY);
                dn = std::nextafter(dn, -INFINITY);
                cj[1 + 2 * k] = up;
                cj[2 + 2 * k] = dn;
            }
            ok = advance(j);
        }
        // every entry, bitwise (rows in parallel); columns that fail move on to
        // their next candidate, a few rounds at most
        for (int round = 0; ok && round < kC; ++round) {
            // (atomic flags: a column is counted once, on its 0 -> 1 transition)
            std::unique_ptr<std::atomic<unsigned char>[]> badcol(
                new std::atomic<unsigned char>[w]);
            for (long j = 0; j < w; ++j) badcol[j].store(0, std::memory_order_relaxed);
            std::atomic<long> nbad{0};
            parallel_rows(rows, nthreads, [&](long r0, long r1) {
                for (long i = r0; i < r1; ++i) {
                    const double *row = v + i * ld;
                    for (long j = 0; j < w; ++j)
                        if (bits(a[i] * b[j]) != bits(row[j]) &&
                            !badcol[j].load(std::memory_order_relaxed) &&
                            !badcol[j].exchange(1, std::memory_order_relaxed))
                            nbad++;
                    if (nbad.load(std::memory_order_relaxed) > w / 4 + 8) return;
                }
            });
            if (nbad == 0) break;
            if (nbad > w / 4 + 8) {
                ok = false;
                break;
            }
            for (long j = 0; j < w && ok; ++j)
                if (badcol[j]) ok = advance(j);
            if (round == kC - 1) ok = false;
        }
        if (!ok) continue;
        // nonzero magnitudes must stay normal after the scalings by h/2 >= smin
        if (smin > 0) {
            for (long j = 0; j < w; ++j)
                if (b[j] != 0.0 && std::fabs(b[j]) * smin < DBL_MIN) return false;
            std::atomic<bool> rng{true};
            parallel_rows(rows, nthreads, [&](long r0, long r1) {
                for (long i = r0; i < r1; ++i)
                    for (long j = 0; j < w; ++j) {
                        const double x = v[i * ld + j];
                        if (x != 0.0 && std::fabs(x) * smin < DBL_MIN) {
                            rng = false;
                            return;
                        }
                    }
            });
            if (!rng) return false;
        }
        if (jsel) *jsel = js;
        return true;
    }
    return false;
}

}  // namespace mgxsep
