/* mg_oracle.c -- CPU restatement of the reference geometric-multigrid path.
 *
 * TEST INFRASTRUCTURE ONLY (see mg_oracle.h).  Never linked into the product.
 *
 * Every function restates one reference function with the same floating-point
 * term order, so that on x86-64 (SSE2 doubles, no FMA contraction: the Makefile
 * builds with -ffp-contract=off) results are bitwise equal to the reference
 * compiled with its own Makefile flags.  Differences from the reference are
 * limited to things that cannot change a value:
 *   - 64-bit index arithmetic everywhere (the reference overflows int for
 *     (N+1)^2 > 2^31);
 *   - the red (resp. black) points of gauss_seidel are visited row by row
 *     instead of "odd rows then even rows"; updates of one colour read only
 *     the other colour, so the visiting order is irrelevant;
 *   - coarse tower buffers are zero-filled (calloc), which pins the
 *     reference's uninitialised-memory read.
 */
#include "mg_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static int g_threads = 1;

void or_set_threads(int nthreads) { g_threads = nthreads < 1 ? 1 : nthreads; }

/* fp_mode fma (libmgx stencil.h): 0 = the reference's expressions */
static int g_fm = 0;
void or_set_fp_mode(int fm) { g_fm = fm ? 1 : 0; }

/* The fma form's constants, as libmgx's make_coef computes them on the host
 * (kernels.hip): d = 1-4 rr nu, rd = 1/d, g = rr/d, gn = g nu, c2 = -2 gn. */
typedef struct {
    double dgs, rdgs, g, gn, c2, hh;
} FmCoef;
static FmCoef fm_coef(double k, double nu, double h) {
    FmCoef f;
    const double rr = 0.5 * k / (h * h);
    f.dgs = 1.0 - 4.0 * rr * nu;
    f.rdgs = 1.0 / f.dgs;
    f.g = rr / f.dgs;
    f.gn = f.g * nu;
    f.c2 = -2.0 * f.gn;
    f.hh = h * 0.5;
    return f;
}
/* u = f/d + mn uN + mw uW + me uE + ms uS as libmgx evaluates it: t = v*h/2,
 * mn = fma(g, t1, -gn), mw = fma(g, t2, -gn), ms = c2 - mn, me = c2 - mw,
 * the fmas in the order N, W, E, S */
static inline double fm_update(const FmCoef *f, double rhs, double v1, double v2, double uN,
                               double uW, double uS, double uE) {
    const double fs = rhs * f->rdgs;
    const double mn = fma(f->g, v1 * f->hh, -f->gn), mw = fma(f->g, v2 * f->hh, -f->gn);
    const double ms = f->c2 - mn, me = f->c2 - mw;
    return fma(ms, uS, fma(me, uE, fma(mw, uW, fma(mn, uN, fs))));
}

/* gs.cpp:9-11 */
static inline double coef_r(double h, double k) { return 0.5 * k / (h * h); }
/* gs.cpp:14-16 */
static inline double coef_a(double v, double nu, double h, double r) {
    return r * (-v * h / 2.0 + nu);
}
/* gs.cpp:18-20 */
static inline double coef_b(double v, double nu, double h, double r) {
    return r * (v * h / 2.0 + nu);
}

/* gs.cpp:24-53.  rhs = (1+4 r nu) u - cc uN - aa uW - dd uS - bb uE (gs.cpp:44). */
void or_compute_rhs(double *rhs, const double *u, long n, const double *v1,
                    const double *v2, double k, double nu, double h) {
    const double rr = coef_r(h, k);
    const long w = n + 1;
#pragma omp parallel for schedule(static) if (g_threads > 1) num_threads(g_threads)
    for (long i = 1; i < n; i++) {
        for (long j = 1; j < n; j++) {
            const long p = i * w + j;
            const double aa = coef_a(v2[p], nu, h, rr);
            const double bb = coef_b(v2[p], nu, h, rr);
            const double cc = coef_a(v1[p], nu, h, rr);
            const double dd = coef_b(v1[p], nu, h, rr);
            rhs[p] = (1.0 + 4.0 * rr * nu) * u[p] - cc * u[p - w] - aa * u[p - 1] -
                     dd * u[p + w] - bb * u[p + 1];
        }
    }
}

/* gs.cpp:55-83.  Interior only; the boundary of res is left untouched. */
void or_residual(double *res, const double *u, const double *rhs, long n,
                 const double *v1, const double *v2, double k, double nu, double h) {
    const double rr = coef_r(h, k);
    const long w = n + 1;
    if (g_fm) { /* libmgx fp_mode fma: d*(update - u) */
        const FmCoef f = fm_coef(k, nu, h);
#pragma omp parallel for schedule(static) if (g_threads > 1) num_threads(g_threads)
        for (long i = 1; i < n; i++)
            for (long j = 1; j < n; j++) {
                const long p = i * w + j;
                res[p] = (fm_update(&f, rhs[p], v1[p], v2[p], u[p - w], u[p - 1], u[p + w],
                                    u[p + 1]) - u[p]) * f.dgs;
            }
        return;
    }
#pragma omp parallel for schedule(static) if (g_threads > 1) num_threads(g_threads)
    for (long i = 1; i < n; i++) {
        for (long j = 1; j < n; j++) {
            const long p = i * w + j;
            const double aa = coef_a(v2[p], nu, h, rr);
            const double bb = coef_b(v2[p], nu, h, rr);
            const double cc = coef_a(v1[p], nu, h, rr);
            const double dd = coef_b(v1[p], nu, h, rr);
            res[p] = rhs[p] - ((1.0 - 4.0 * rr * nu) * u[p] + cc * u[p - w] +
                               aa * u[p - 1] + dd * u[p + w] + bb * u[p + 1]);
        }
    }
}

/* gs.cpp:86-107.  Serial row-major accumulation of the interior squares. */
double or_compute_norm(const double *res, long n) {
    double acc = 0.0;
    const long w = n + 1;
    for (long i = 1; i < n; i++)
        for (long j = 1; j < n; j++) acc += res[i * w + j] * res[i * w + j];
    return sqrt(acc);
}

/* One colour of gs.cpp:109-189: colour 0 = red = (i+j) even (gs.cpp:121-151),
 * colour 1 = black = (i+j) odd (gs.cpp:156-184).  Update term order gs.cpp:130. */
static void gs_colour(double *u, const double *rhs, long n, const double *v1,
                      const double *v2, double k, double nu, double h, int colour) {
    const double rr = coef_r(h, k);
    const long w = n + 1;
    if (g_fm) { /* libmgx fp_mode fma */
        const FmCoef f = fm_coef(k, nu, h);
#pragma omp parallel for schedule(static) if (g_threads > 1) num_threads(g_threads)
        for (long i = 1; i < n; i++) {
            const long j0 = (colour == 0) ? (2 - (i & 1)) : (1 + (i & 1));
            for (long j = j0; j < n; j += 2) {
                const long p = i * w + j;
                u[p] = fm_update(&f, rhs[p], v1[p], v2[p], u[p - w], u[p - 1], u[p + w],
                                 u[p + 1]);
            }
        }
        return;
    }
#pragma omp parallel for schedule(static) if (g_threads > 1) num_threads(g_threads)
    for (long i = 1; i < n; i++) {
        /* red: odd rows start at j=1, even rows at j=2; black the opposite */
        const long j0 = (colour == 0) ? (2 - (i & 1)) : (1 + (i & 1));
        for (long j = j0; j < n; j += 2) {
            const long p = i * w + j;
            const double aa = coef_a(v2[p], nu, h, rr);
            const double bb = coef_b(v2[p], nu, h, rr);
            const double cc = coef_a(v1[p], nu, h, rr);
            const double dd = coef_b(v1[p], nu, h, rr);
            u[p] = (rhs[p] - cc * u[p - w] - aa * u[p - 1] - dd * u[p + w] -
                    bb * u[p + 1]) /
                   (1.0 - 4.0 * rr * nu);
        }
    }
}

void or_gauss_seidel(double *u, const double *rhs, long n, const double *v1,
                     const double *v2, double k, double nu, double h) {
    gs_colour(u, rhs, n, v1, v2, k, nu, h, 0);
    gs_colour(u, rhs, n, v1, v2, k, nu, h, 1);
}

/* gs.cpp:228-266.  up: (2n+1)^2 output, u: (n+1)^2 input; bilinear. */
void or_prolongation(double *up, const double *u, long n) {
    const long w = n + 1, W = 2 * n + 1;
#pragma omp parallel for schedule(static) if (g_threads > 1) num_threads(g_threads)
    for (long i = 0; i < n; i++) {
        for (long j = 0; j < n; j++) {
            up[2 * i * W + 2 * j] = u[i * w + j];
            up[(2 * i + 1) * W + 2 * j] = (u[i * w + j] + u[(i + 1) * w + j]) / 2;
            up[2 * i * W + 2 * j + 1] = (u[i * w + j] + u[i * w + j + 1]) / 2;
            up[(2 * i + 1) * W + 2 * j + 1] = (u[i * w + j] + u[(i + 1) * w + j] +
                                               u[i * w + j + 1] + u[(i + 1) * w + j + 1]) / 4;
        }
    }
    /* right and bottom borders (gs.cpp:251-260) */
    for (long i = 0; i < n; i++) {
        up[2 * i * W + 2 * n] = u[i * w + n];
        up[(2 * i + 1) * W + 2 * n] = (u[i * w + n] + u[(i + 1) * w + n]) / 2;
        up[2 * n * W + 2 * i] = u[n * w + i];
        up[2 * n * W + 2 * i + 1] = (u[n * w + i] + u[n * w + i + 1]) / 2;
    }
    up[2 * n * W + 2 * n] = u[n * w + n]; /* gs.cpp:265 */
}

/* gs.cpp:268-292.  Injection including the boundary: u is (n/2+1)^2 output,
 * up is read as an (n+1)-wide array (gs.cpp:283). */
void or_restriction(double *u, const double *up, long n) {
    const long m = n / 2 + 1, w = n + 1;
#pragma omp parallel for schedule(static) if (g_threads > 1) num_threads(g_threads)
    for (long i = 0; i < m; i++)
        for (long j = 0; j < m; j++) u[i * m + j] = up[2 * i * w + 2 * j];
}

/* multigrid.cpp:17-92 */
long or_mg_inner(double **u, double **rhs, double **v1, double **v2, double *tmp,
                 double dx, long n, int lvl, int maxlvl, int shape, double dt,
                 double nu, int nsmooth) {
    long coarse_iters = 0;
    double *ui = u[lvl], *rhsi = rhs[lvl], *v1i = v1[lvl], *v2i = v2[lvl];
    const long nnew = n / 2;
    const double dx2 = 2 * dx;
    for (int sh = 0; sh < shape; ++sh) {
        if (lvl == maxlvl - 1) {
            /* coarsest level: GS until |res| <= 1e-5 or 1000 sweeps (:58-65) */
            double res_exact = 1.0;
            int i = 0;
            while (i < 1000 && res_exact > 1e-5) {
                or_gauss_seidel(ui, rhsi, n, v1i, v2i, dt, nu, dx);
                or_residual(tmp, ui, rhsi, n, v1i, v2i, dt, nu, dx);
                res_exact = or_compute_norm(tmp, n);
                i++;
            }
            coarse_iters += i;
        } else {
            double *ui1 = u[lvl + 1], *rhsi1 = rhs[lvl + 1];
            for (int it = 0; it < nsmooth; ++it)
                or_gauss_seidel(ui, rhsi, n, v1i, v2i, dt, nu, dx);
            or_residual(tmp, ui, rhsi, n, v1i, v2i, dt, nu, dx);
            or_restriction(rhsi1, tmp, n);
            memset(ui1, 0, sizeof(double) * (size_t)(nnew + 1) * (size_t)(nnew + 1));
            coarse_iters += or_mg_inner(u, rhs, v1, v2, tmp, dx2, nnew, lvl + 1, maxlvl,
                                        shape, dt, nu, nsmooth);
            or_prolongation(tmp, ui1, nnew);
            const long tot = (n + 1) * (n + 1);
            for (long p = 0; p < tot; ++p) ui[p] += tmp[p];
            for (int it = 0; it < nsmooth; ++it)
                or_gauss_seidel(ui, rhsi, n, v1i, v2i, dt, nu, dx);
        }
    }
    return coarse_iters;
}

/* multigrid.cpp:94-120 */
int or_mg_outer(double **utow, double **v1tow, double **v2tow, double **rhstow,
                double *tmp, double nu, int maxlvl, long n, double dt, double dx,
                double tol, int shape, int nsmooth, double *res0_out,
                double *res_out) {
    const int max_cycle = 50; /* multigrid.cpp:94 */
    const int fm = g_fm; /* (libmgx's initial norm is the reference's residual) */
    g_fm = 0;
    or_residual(tmp, utow[0], rhstow[0], n, v1tow[0], v2tow[0], dt, nu, dx);
    g_fm = fm;
    double res0 = or_compute_norm(tmp, n), res = res0;
    int iter;
    for (iter = 0; iter < max_cycle && res / res0 > tol; iter++) {
        or_mg_inner(utow, rhstow, v1tow, v2tow, tmp, dx, n, 0, maxlvl, shape, dt, nu,
                    nsmooth);
        or_residual(tmp, utow[0], rhstow[0], n, v1tow[0], v2tow[0], dt, nu, dx);
        res = or_compute_norm(tmp, n);
    }
    if (res0_out) *res0_out = res0;
    if (res_out) *res_out = res;
    return iter;
}

/* multigrid.cpp:148-160 (REFERENCE mode reproduces its index quirk, K2). */
void or_build_tower(double **v1tow, double **v2tow, double **utow, double **rhstow,
                    int maxlvl, long n, int tower_mode) {
    for (int i = 1; i < maxlvl; i++) {
        long ni, nsrc;
        if (tower_mode == OR_TOWER_REFERENCE) {
            ni = (n >> 1) + 1; /* multigrid.cpp:150: same size on every level */
            nsrc = ni - 1;     /* multigrid.cpp:155: restriction(.., .., ni-1) */
        } else {
            ni = (n >> i) + 1;
            nsrc = n >> (i - 1);
        }
        const size_t cnt = (size_t)ni * (size_t)ni;
        utow[i] = (double *)calloc(cnt, sizeof(double));
        v1tow[i] = (double *)calloc(cnt, sizeof(double));
        v2tow[i] = (double *)calloc(cnt, sizeof(double));
        rhstow[i] = (double *)calloc(cnt, sizeof(double));
        or_restriction(v1tow[i], v1tow[i - 1], nsrc);
        or_restriction(v2tow[i], v2tow[i - 1], nsrc);
    }
}

void or_free_tower(double **v1tow, double **v2tow, double **utow, double **rhstow,
                   int maxlvl) {
    for (int i = 1; i < maxlvl; i++) {
        free(utow[i]);
        free(v1tow[i]);
        free(v2tow[i]);
        free(rhstow[i]);
    }
}

/* multigrid.cpp:124-186 */
int or_timestepper(double *uT, const double *u0, const double *v1, const double *v2,
                   double nu, int maxlvl, long n, double dt, double T, double dx,
                   double tol, int shape, int nsmooth, int tower_mode,
                   int *cycles_per_step) {
    double **utow = (double **)calloc((size_t)maxlvl + 1, sizeof(double *));
    double **v1tow = (double **)calloc((size_t)maxlvl + 1, sizeof(double *));
    double **v2tow = (double **)calloc((size_t)maxlvl + 1, sizeof(double *));
    double **rhstow = (double **)calloc((size_t)maxlvl + 1, sizeof(double *));
    const size_t cnt = (size_t)(n + 1) * (size_t)(n + 1);
    utow[0] = (double *)malloc(cnt * sizeof(double));
    v1tow[0] = (double *)malloc(cnt * sizeof(double));
    v2tow[0] = (double *)malloc(cnt * sizeof(double));
    rhstow[0] = (double *)calloc(cnt, sizeof(double));
    memcpy(utow[0], u0, cnt * sizeof(double));
    memcpy(v1tow[0], v1, cnt * sizeof(double));
    memcpy(v2tow[0], v2, cnt * sizeof(double));
    or_build_tower(v1tow, v2tow, utow, rhstow, maxlvl, n, tower_mode);
    double *tmp = (double *)calloc(cnt, sizeof(double));

    const int steps = (int)(T / dt); /* multigrid.cpp:165 */
    for (int it = 0; it < steps; it++) {
        or_compute_rhs(rhstow[0], utow[0], n, v1tow[0], v2tow[0], dt, nu, dx);
        int cyc = or_mg_outer(utow, v1tow, v2tow, rhstow, tmp, nu, maxlvl, n, dt, dx,
                              tol, shape, nsmooth, NULL, NULL);
        if (cycles_per_step) cycles_per_step[it] = cyc;
    }
    memcpy(uT, utow[0], cnt * sizeof(double));

    free(tmp);
    or_free_tower(v1tow, v2tow, utow, rhstow, maxlvl);
    free(utow[0]);
    free(v1tow[0]);
    free(v2tow[0]);
    free(rhstow[0]);
    free(utow);
    free(v1tow);
    free(v2tow);
    free(rhstow);
    return steps;
}

/* multigrid.cpp:206-233 */
void or_init_problem(double *u0, double *v1, double *v2, long N) {
    const double PI = 3.1415926535897932; /* multigrid.cpp:14 */
    const double dx = 1.0 / N;
    const double x0 = 0.2, y0 = 0.4, sigma = 100.0, kx = 1.0 * PI, ky = 1.0 * PI;
    const long w = N + 1;
#pragma omp parallel for schedule(static) if (g_threads > 1) num_threads(g_threads)
    for (long i = 0; i < w; ++i) {
        for (long j = 0; j < w; ++j) {
            /* the reference multiplies an int by dx: i*dx converts i exactly */
            const double xi = (double)i, yj = (double)j;
            u0[i * w + j] = exp(-sigma * ((xi * dx - x0) * (xi * dx - x0) +
                                          (yj * dx - y0) * (yj * dx - y0)));
            v1[i * w + j] = -ky * sin(kx * xi * dx) * cos(ky * yj * dx);
            v2[i * w + j] = kx * cos(kx * xi * dx) * sin(ky * yj * dx);
        }
    }
    /* zero boundary (multigrid.cpp:227-233) */
    for (long i = 0; i < N; ++i) {
        u0[i] = 0.0;
        u0[i * w + N] = 0.0;
        u0[N * w + i + 1] = 0.0;
        u0[i * w] = 0.0;
    }
}

/* ---------------------------------------------------------------- row slabs
 * The gs.h ops on a window of rows: the arrays hold global rows [r0, r0+nr)
 * of an (n+1)^2 field (row-major, width n+1), so a test can check the device
 * ops at sizes where the whole field does not fit the host (N = 65536: 4.3e9
 * points per array).  Same expressions and term order as the
 * whole-field functions above; only points whose stencil lies inside the
 * window are updated: a slab result is the whole-field result on rows
 * [r0+1, r0+nr-2] (residual / compute_rhs) and [r0+2, r0+nr-3] (gauss_seidel,
 * whose black half reads red values one row further out). */
static void slab_rows(long n, long r0, long nr, long *i0, long *i1) {
    *i0 = r0 + 1 > 1 ? r0 + 1 : 1;
    *i1 = r0 + nr - 1 < n ? r0 + nr - 1 : n; /* exclusive */
}

/* gs.cpp:109-189 on a slab */
void or_gauss_seidel_slab(double *u, const double *rhs, long n, long r0, long nr,
                          const double *v1, const double *v2, double k, double nu, double h) {
    const double rr = coef_r(h, k);
    const long w = n + 1;
    long i0, i1;
    slab_rows(n, r0, nr, &i0, &i1);
    for (int colour = 0; colour < 2; colour++) {
#pragma omp parallel for schedule(static) if (g_threads > 1) num_threads(g_threads)
        for (long i = i0; i < i1; i++) {
            const long j0 = (colour == 0) ? (2 - (i & 1)) : (1 + (i & 1));
            for (long j = j0; j < n; j += 2) {
                const long p = (i - r0) * w + j;
                const double aa = coef_a(v2[p], nu, h, rr);
                const double bb = coef_b(v2[p], nu, h, rr);
                const double cc = coef_a(v1[p], nu, h, rr);
                const double dd = coef_b(v1[p], nu, h, rr);
                u[p] = (rhs[p] - cc * u[p - w] - aa * u[p - 1] - dd * u[p + w] -
                        bb * u[p + 1]) /
                       (1.0 - 4.0 * rr * nu);
            }
        }
    }
}

/* gs.cpp:55-83 on a slab */
void or_residual_slab(double *res, const double *u, const double *rhs, long n, long r0,
                      long nr, const double *v1, const double *v2, double k, double nu,
                      double h) {
    const double rr = coef_r(h, k);
    const long w = n + 1;
    long i0, i1;
    slab_rows(n, r0, nr, &i0, &i1);
#pragma omp parallel for schedule(static) if (g_threads > 1) num_threads(g_threads)
    for (long i = i0; i < i1; i++) {
        for (long j = 1; j < n; j++) {
            const long p = (i - r0) * w + j;
            const double aa = coef_a(v2[p], nu, h, rr);
            const double bb = coef_b(v2[p], nu, h, rr);
            const double cc = coef_a(v1[p], nu, h, rr);
            const double dd = coef_b(v1[p], nu, h, rr);
            res[p] = rhs[p] - ((1.0 - 4.0 * rr * nu) * u[p] + cc * u[p - w] +
                               aa * u[p - 1] + dd * u[p + w] + bb * u[p + 1]);
        }
    }
}

/* gs.cpp:24-53 on a slab */
void or_compute_rhs_slab(double *rhs, const double *u, long n, long r0, long nr,
                         const double *v1, const double *v2, double k, double nu, double h) {
    const double rr = coef_r(h, k);
    const long w = n + 1;
    long i0, i1;
    slab_rows(n, r0, nr, &i0, &i1);
#pragma omp parallel for schedule(static) if (g_threads > 1) num_threads(g_threads)
    for (long i = i0; i < i1; i++) {
        for (long j = 1; j < n; j++) {
            const long p = (i - r0) * w + j;
            const double aa = coef_a(v2[p], nu, h, rr);
            const double bb = coef_b(v2[p], nu, h, rr);
            const double cc = coef_a(v1[p], nu, h, rr);
            const double dd = coef_b(v1[p], nu, h, rr);
            rhs[p] = (1.0 + 4.0 * rr * nu) * u[p] - cc * u[p - w] - aa * u[p - 1] -
                     dd * u[p + w] - bb * u[p + 1];
        }
    }
}

/* gs.cpp:228-266 for fine rows [2 c0, 2 (c0 + cn - 1)] (clipped to 2n) from
 * coarse rows [c0, c0 + cn): up holds those fine rows (width 2n+1).  The
 * interior formulas (gs.cpp:238-241) and the border ones (gs.cpp:251-265) are
 * the same expressions at i = n or j = n, evaluated per fine point here. */
void or_prolongation_slab(double *up, const double *u, long n, long c0, long cn) {
    const long w = n + 1, W = 2 * n + 1;
    long I1 = 2 * (c0 + cn - 1);
    if (I1 > 2 * n) I1 = 2 * n;
#pragma omp parallel for schedule(static) if (g_threads > 1) num_threads(g_threads)
    for (long I = 2 * c0; I <= I1; I++) {
        const long i = I >> 1;
        const double *r0 = u + (i - c0) * w;
        for (long J = 0; J < W; J++) {
            const long j = J >> 1;
            double v;
            if (!(I & 1))
                v = (J & 1) ? (r0[j] + r0[j + 1]) / 2 : r0[j];
            else if (!(J & 1))
                v = (r0[j] + r0[w + j]) / 2;
            else
                v = (r0[j] + r0[w + j] + r0[j + 1] + r0[w + j + 1]) / 4;
            up[(I - 2 * c0) * W + J] = v;
        }
    }
}
