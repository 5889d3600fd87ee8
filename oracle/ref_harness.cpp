// ref_harness.cpp -- C entry points around the UNMODIFIED reference sources.
//
// TEST INFRASTRUCTURE ONLY.  oracle/Makefile compiles /root/reference/gs.cpp and
// /root/reference/multigrid.cpp (with -Dmain=mg_reference_main, Makefile flags
// -O0 -fopenmp -std=c++11) together with this file into oracle/_ref/libmgref.so.
// Nothing of the reference is copied here: the prototypes below are the
// reference's own signatures (gs.h:3-17, multigrid.cpp:17,97,124) so that the
// linker binds them to the reference objects.
//
// Uses: pinning the C restatement (tests/test_oracle_pin.py), generating the
// golden fixtures (tests/golden/make_golden.py) and the cpu_baseline leg of
// bench.py (kind "reference").
#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>

#include "gs.h"  // from /root/reference via -I

// multigrid.cpp:17, :97, :124 (C++ linkage, defined in the reference object)
void mg_inner(double **u, double **rhs, double **v1, double **v2, double *tmp, double dx,
              int n, int lvl, int maxlvl, int shape, double dt, double nu);
void mg_outer(double **utow, double **v1tow, double **v2tow, double **rhstow, double *tmp,
              double nu, int maxlvl, int n, double dt, double dx, double tol, int shape);
void timestepper(double *uT, double *u0, double *v1, double *v2, double nu, int maxlvl,
                 int n, double dt, double T, double dx, double tol, int shape);

namespace {

// The reference's gs.cpp ops spawn orphaned `omp task`s; they only fan out when
// called from inside `omp parallel` + `single` (multigrid.cpp:252-258).
template <class F>
void run_threads(int nthreads, F &&f) {
    if (nthreads <= 1) {
        f();
        return;
    }
#pragma omp parallel num_threads(nthreads)
    {
#pragma omp single
        { f(); }
    }
}

struct Tower {
    int maxlvl = 0;
    double **u = nullptr, **rhs = nullptr, **v1 = nullptr, **v2 = nullptr;
    double *tmp = nullptr;
};

// Same construction as timestepper (multigrid.cpp:138-162), with calloc for the
// coarse levels (the reference's malloc'd coarse buffers are read
// before being written; zero-fill is the pinned semantics).  correct = 1: the
// CORRECT tower instead (SURVEY K2's fix, mgx's MGX_TOWER_CORRECT): level i is
// ((n >> i) + 1)^2 and the reference's own restriction of level i-1 at its
// true size n >> (i-1); mg_inner then reads every level at the width it was
// built with.
void build(Tower &t, const double *u0, const double *v1, const double *v2, int maxlvl, int n,
           int correct = 0) {
    t.maxlvl = maxlvl;
    t.u = (double **)calloc(maxlvl + 1, sizeof(double *));
    t.rhs = (double **)calloc(maxlvl + 1, sizeof(double *));
    t.v1 = (double **)calloc(maxlvl + 1, sizeof(double *));
    t.v2 = (double **)calloc(maxlvl + 1, sizeof(double *));
    size_t cnt = (size_t)(n + 1) * (n + 1);
    t.u[0] = (double *)malloc(cnt * sizeof(double));
    t.v1[0] = (double *)malloc(cnt * sizeof(double));
    t.v2[0] = (double *)malloc(cnt * sizeof(double));
    t.rhs[0] = (double *)calloc(cnt, sizeof(double));
    memcpy(t.u[0], u0, cnt * sizeof(double));
    memcpy(t.v1[0], v1, cnt * sizeof(double));
    memcpy(t.v2[0], v2, cnt * sizeof(double));
    for (int i = 1; i < maxlvl; i++) {
        int ni = correct ? (n >> i) + 1 : (n >> 1) + 1;
        int nr = correct ? n >> (i - 1) : ni - 1;   // the `n` restriction is passed
        t.u[i] = (double *)calloc((size_t)ni * ni, sizeof(double));
        t.v1[i] = (double *)calloc((size_t)ni * ni, sizeof(double));
        restriction(t.v1[i], t.v1[i - 1], nr);
        t.v2[i] = (double *)calloc((size_t)ni * ni, sizeof(double));
        restriction(t.v2[i], t.v2[i - 1], nr);
        t.rhs[i] = (double *)calloc((size_t)ni * ni, sizeof(double));
    }
    t.tmp = (double *)calloc(cnt, sizeof(double));
}

void release(Tower &t) {
    for (int i = 0; i < t.maxlvl; i++) {
        free(t.u[i]);
        free(t.rhs[i]);
        free(t.v1[i]);
        free(t.v2[i]);
    }
    free(t.u);
    free(t.rhs);
    free(t.v1);
    free(t.v2);
    free(t.tmp);
}

}  // namespace

extern "C" {

void ref_gauss_seidel(double *u, double *rhs, long n, double *v1, double *v2, double k,
                      double nu, double h, int nthreads) {
    run_threads(nthreads, [&] { gauss_seidel(u, rhs, n, v1, v2, k, nu, h); });
}
void ref_residual(double *res, double *u, double *rhs, long n, double *v1, double *v2,
                  double k, double nu, double h) {
    residual(res, u, rhs, n, v1, v2, k, nu, h);
}
double ref_compute_norm(double *res, long n) { return compute_norm(res, n); }
void ref_prolongation(double *up, double *u, int n) { prolongation(up, u, n); }
void ref_restriction(double *u, double *up, int n) { restriction(u, up, n); }
void ref_compute_rhs(double *rhs, double *u, long n, double *v1, double *v2, double k,
                     double nu, double h) {
    compute_rhs(rhs, u, n, v1, v2, k, nu, h);
}

// The library is linked with -Wl,--wrap=malloc: every malloc in the reference
// objects lands here and returns zero-filled memory.  timestepper mallocs its
// coarse towers and reads parts of them before writing them; the
// zero fill pins that read, independent of the state of the process heap.
void *__wrap_malloc(size_t bytes) { return calloc(1, bytes); }

// The reference timestepper, unmodified.
void ref_timestepper(double *uT, double *u0, double *v1, double *v2, double nu, int maxlvl,
                     int n, double dt, double T, double dx, double tol, int shape,
                     int nthreads) {
    run_threads(nthreads,
                [&] { timestepper(uT, u0, v1, v2, nu, maxlvl, n, dt, T, dx, tol, shape); });
}

// One reference V-cycle (mg_inner) on a fresh tower built from (u, v1, v2) with
// rhs = compute_rhs(u) (multigrid.cpp:167); u is updated in place.  Returns the
// norm of the residual after the cycle (multigrid.cpp:112-113).
double ref_vcycle_once_tower(double *u, double *v1, double *v2, int n, int maxlvl, double dt,
                             double nu, int shape, int nthreads, int correct) {
    Tower t;
    build(t, u, v1, v2, maxlvl, n, correct);
    double dx = 1.0 / n, res = 0.0;
    run_threads(nthreads, [&] {
        compute_rhs(t.rhs[0], t.u[0], n, t.v1[0], t.v2[0], dt, nu, dx);
        mg_inner(t.u, t.rhs, t.v1, t.v2, t.tmp, dx, n, 0, maxlvl, shape, dt, nu);
        residual(t.tmp, t.u[0], t.rhs[0], n, t.v1[0], t.v2[0], dt, nu, dx);
        res = compute_norm(t.tmp, n);
    });
    memcpy(u, t.u[0], (size_t)(n + 1) * (n + 1) * sizeof(double));
    release(t);
    return res;
}
double ref_vcycle_once(double *u, double *v1, double *v2, int n, int maxlvl, double dt,
                       double nu, int shape, int nthreads) {
    return ref_vcycle_once_tower(u, v1, v2, n, maxlvl, dt, nu, shape, nthreads, 0);
}

// CPU baseline: `cycles` timed V-cycles (mg_inner + residual + compute_norm, the
// bench step of SURVEY 8d) of the reference problem at size n, after rhs setup.
// Returns wall seconds for the timed cycles; *setup_s gets the untimed setup.
double ref_time_vcycles(int n, int maxlvl, double nu, int cycles, int nthreads,
                        double *setup_s, double *final_res) {
    double t0 = omp_get_wtime();
    // the untimed setup uses every host thread, whatever `nthreads` the timed
    // cycles get (a serial -O0 init of N=16384 alone takes longer than the cycle)
    const int setup_threads = omp_get_num_procs() > nthreads ? omp_get_num_procs() : nthreads;
    size_t cnt = (size_t)(n + 1) * (n + 1);
    double *u0 = (double *)malloc(cnt * sizeof(double));
    double *v1 = (double *)malloc(cnt * sizeof(double));
    double *v2 = (double *)malloc(cnt * sizeof(double));
    const double PI = 3.1415926535897932, dx = 1.0 / n;
#pragma omp parallel for num_threads(setup_threads > 0 ? setup_threads : 1)
    for (long i = 0; i < n + 1; ++i)
        for (long j = 0; j < n + 1; ++j) {
            u0[i * (n + 1) + j] = exp(-100.0 * ((i * dx - 0.2) * (i * dx - 0.2) +
                                                 (j * dx - 0.4) * (j * dx - 0.4)));
            v1[i * (n + 1) + j] = -PI * sin(PI * i * dx) * cos(PI * j * dx);
            v2[i * (n + 1) + j] = PI * cos(PI * i * dx) * sin(PI * j * dx);
        }
    for (long i = 0; i < n; ++i) {
        u0[i] = 0.0;
        u0[i * (n + 1) + n] = 0.0;
        u0[(long)n * (n + 1) + i + 1] = 0.0;
        u0[i * (n + 1)] = 0.0;
    }
    Tower t;
    build(t, u0, v1, v2, maxlvl, n);
    free(u0);
    free(v1);
    free(v2);
    double dt = dx / 10, res = 0.0;
    run_threads(setup_threads, [&] { compute_rhs(t.rhs[0], t.u[0], n, t.v1[0], t.v2[0], dt, nu, dx); });
    double t1 = omp_get_wtime();
    run_threads(nthreads, [&] {
        for (int c = 0; c < cycles; ++c) {
            mg_inner(t.u, t.rhs, t.v1, t.v2, t.tmp, dx, n, 0, maxlvl, 1, dt, nu);
            residual(t.tmp, t.u[0], t.rhs[0], n, t.v1[0], t.v2[0], dt, nu, dx);
            res = compute_norm(t.tmp, n);
        }
    });
    double t2 = omp_get_wtime();
    release(t);
    if (setup_s) *setup_s = t1 - t0;
    if (final_res) *final_res = res;
    return t2 - t1;
}

}  // extern "C"
