/* mg_oracle.h -- CPU restatement of the reference multigrid path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline).  The product (hpcclassmultigridproject_amd,
 * libmgx.so, driver/) never links or calls it.
 *
 * Pinned against the reference itself: oracle/Makefile builds the unmodified
 * /root/reference/{gs,multigrid}.cpp into oracle/_ref/libmgref.so and
 * tests/test_oracle_pin.py checks this restatement bitwise against it; the
 * committed fixtures under tests/golden/ were produced by that build
 * (tests/golden/make_golden.py).
 *
 * Layout: level arrays are row-major (n+1)*(n+1) doubles, element (i,j) at
 * i*(n+1)+j, exactly as gs.cpp:44 etc.
 */
#ifndef MG_ORACLE_H
#define MG_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* gs.cpp:24-53 */
void or_compute_rhs(double *rhs, const double *u, long n, const double *v1,
                    const double *v2, double k, double nu, double h);
/* gs.cpp:55-83 */
void or_residual(double *res, const double *u, const double *rhs, long n,
                 const double *v1, const double *v2, double k, double nu, double h);
/* gs.cpp:86-107 */
double or_compute_norm(const double *res, long n);
/* gs.cpp:109-189 (nthreads>1: rows of one colour split over OpenMP threads) */
void or_gauss_seidel(double *u, const double *rhs, long n, const double *v1,
                     const double *v2, double k, double nu, double h);
/* gs.cpp:228-266 */
void or_prolongation(double *up, const double *u, long n);
/* gs.cpp:268-292 */
void or_restriction(double *u, const double *up, long n);
/* Row-slab forms (arrays hold global rows [r0, r0+nr) of an (n+1)^2 field),
 * for checking the device ops at N where a field does not fit the host. */
void or_gauss_seidel_slab(double *u, const double *rhs, long n, long r0, long nr,
                          const double *v1, const double *v2, double k, double nu, double h);
void or_residual_slab(double *res, const double *u, const double *rhs, long n, long r0,
                      long nr, const double *v1, const double *v2, double k, double nu,
                      double h);
void or_compute_rhs_slab(double *rhs, const double *u, long n, long r0, long nr,
                         const double *v1, const double *v2, double k, double nu, double h);
void or_prolongation_slab(double *up, const double *u, long n, long c0, long cn);

/* multigrid.cpp:17-92.  nsmooth = NITER (multigrid.cpp:41, 3 in the reference).
 * Returns the total number of coarsest-level GS iterations performed. */
long or_mg_inner(double **u, double **rhs, double **v1, double **v2, double *tmp,
                 double dx, long n, int lvl, int maxlvl, int shape, double dt,
                 double nu, int nsmooth);

/* multigrid.cpp:97-120.  Returns the number of V/W-cycles taken; *res_out
 * receives the final residual norm and *res0_out the initial one. */
int or_mg_outer(double **utow, double **v1tow, double **v2tow, double **rhstow,
                double *tmp, double nu, int maxlvl, long n, double dt, double dx,
                double tol, int shape, int nsmooth, double *res0_out,
                double *res_out);

/* Tower modes (multigrid.cpp:148-160). */
#define OR_TOWER_REFERENCE 0 /* coarse buffers (N/2+1)^2, reference index quirk, zero-filled */
#define OR_TOWER_CORRECT 1   /* level l injected from level l-1 with its true width */

/* multigrid.cpp:124-186.  cycles_per_step (may be NULL) receives mg_outer's
 * cycle count for each of the (int)(T/dt) steps. Returns the number of steps. */
int or_timestepper(double *uT, const double *u0, const double *v1, const double *v2,
                   double nu, int maxlvl, long n, double dt, double T, double dx,
                   double tol, int shape, int nsmooth, int tower_mode,
                   int *cycles_per_step);

/* Build the velocity towers the way timestepper does (multigrid.cpp:148-160).
 * v1tow[0]/v2tow[0] must already hold the fine fields; levels 1..maxlvl-1 are
 * allocated here (calloc) and must be released with or_free_tower. */
void or_build_tower(double **v1tow, double **v2tow, double **utow, double **rhstow,
                    int maxlvl, long n, int tower_mode);
void or_free_tower(double **v1tow, double **v2tow, double **utow, double **rhstow,
                   int maxlvl);

/* multigrid.cpp:206-233: Gaussian u0 (x0=.2, y0=.4, sigma=100) with zero
 * boundary, rotating velocity v1=-pi sin(pi x)cos(pi y), v2=pi cos(pi x)sin(pi y). */
void or_init_problem(double *u0, double *v1, double *v2, long N);

/* OpenMP thread count used by the op loops (1 = serial, the default). */
void or_set_threads(int nthreads);
/* 1: gauss_seidel and residual in libmgx's fp_mode fma form (stencil.h "fp_mode
 * fma": the operator divided by its diagonal, four fused multiply-adds per
 * update, residual d*(update - u)) -- a restatement of the product's
 * contracted arithmetic, so the GPU fma mode can be checked bit for bit; 0
 * (default): the reference's term order.  mg_outer's initial norm and
 * compute_rhs stay the reference's in both (as in libmgx). */
void or_set_fp_mode(int fm);

#ifdef __cplusplus
}
#endif
#endif
