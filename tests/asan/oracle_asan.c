/* oracle_asan.c -- AddressSanitizer / UBSan run of the CPU checker
 * (oracle/mg_oracle.c), SURVEY 5 "sanitizer build": every op on exactly-sized
 * heap arrays (so any read or write past an (n+1)^2 field is reported), the
 * slab forms on exactly-sized slabs, both tower modes through the time
 * stepper, W-cycles and the coarsest-level-only case.  Built and run by
 * tests/test_asan.py with -fsanitize=address,undefined.  Test code only. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mg_oracle.h"

static double *field(long n) {
    return (double *)malloc(sizeof(double) * (size_t)(n + 1) * (size_t)(n + 1));
}

static void fill(double *a, long cnt, unsigned seed) {
    for (long i = 0; i < cnt; ++i) {
        seed = seed * 1103515245u + 12345u;
        a[i] = ((seed >> 8) & 0xffff) / 32768.0 - 1.0;
    }
}

static int ops(long n) {
    const double k = 1.0 / n / 10, nu = -4e-4, h = 1.0 / n;
    const long cnt = (n + 1) * (n + 1);
    double *u = field(n), *rhs = field(n), *v1 = field(n), *v2 = field(n), *res = field(n);
    fill(u, cnt, 1);
    fill(rhs, cnt, 2);
    fill(v1, cnt, 3);
    fill(v2, cnt, 4);
    or_compute_rhs(res, u, n, v1, v2, k, nu, h);
    or_residual(res, u, rhs, n, v1, v2, k, nu, h);
    double nr = or_compute_norm(res, n);
    or_gauss_seidel(u, rhs, n, v1, v2, k, nu, h);
    double *up = field(2 * n);
    or_prolongation(up, u, n);
    double *c = field(n / 2);
    or_restriction(c, u, n);
    /* slabs: exactly-sized row windows at the top, middle and bottom */
    const long nr_rows = 6;
    long starts[3] = {0, n / 2 - 3, n + 1 - nr_rows};
    for (int s = 0; s < 3; ++s) {
        const long r0 = starts[s], m = nr_rows * (n + 1);
        double *su = malloc(sizeof(double) * m), *sr = malloc(sizeof(double) * m),
               *s1 = malloc(sizeof(double) * m), *s2 = malloc(sizeof(double) * m),
               *so = malloc(sizeof(double) * m);
        memcpy(su, u + r0 * (n + 1), sizeof(double) * m);
        memcpy(sr, rhs + r0 * (n + 1), sizeof(double) * m);
        memcpy(s1, v1 + r0 * (n + 1), sizeof(double) * m);
        memcpy(s2, v2 + r0 * (n + 1), sizeof(double) * m);
        or_gauss_seidel_slab(su, sr, n, r0, nr_rows, s1, s2, k, nu, h);
        or_residual_slab(so, su, sr, n, r0, nr_rows, s1, s2, k, nu, h);
        or_compute_rhs_slab(so, su, n, r0, nr_rows, s1, s2, k, nu, h);
        const long cr = r0 / 2 + nr_rows / 2 <= n / 2 + 1 ? nr_rows / 2 : 1;
        double *sp = malloc(sizeof(double) * (size_t)(2 * cr) * (2 * (n / 2) + 1));
        or_prolongation_slab(sp, c + (r0 / 2) * (n / 2 + 1), n / 2, r0 / 2,
                             r0 / 2 + cr <= n / 2 + 1 ? cr : n / 2 + 1 - r0 / 2);
        free(sp);
        free(su);
        free(sr);
        free(s1);
        free(s2);
        free(so);
    }
    free(u);
    free(rhs);
    free(v1);
    free(v2);
    free(res);
    free(up);
    free(c);
    return isfinite(nr) ? 0 : 1;
}

static int stepper(long n, int maxlvl, int shape, int tower) {
    double *u0 = field(n), *v1 = field(n), *v2 = field(n), *uT = field(n);
    or_init_problem(u0, v1, v2, n);
    const double dx = 1.0 / n, dt = dx / 10;
    int cyc[3];
    int steps = or_timestepper(uT, u0, v1, v2, -4e-4, maxlvl, n, dt, 3 * dt, dx, 1e-6, shape,
                               3, tower, cyc);
    int bad = steps != 3;
    for (long i = 0; i < (n + 1) * (n + 1); ++i) bad |= !isfinite(uT[i]);
    free(u0);
    free(v1);
    free(v2);
    free(uT);
    return bad;
}

int main(void) {
    int bad = 0;
    long sizes[] = {8, 16, 33 - 1, 64};
    for (int i = 0; i < 4; ++i) bad |= ops(sizes[i]);
    bad |= stepper(32, 1, 1, OR_TOWER_REFERENCE);   /* the coarsest level only */
    bad |= stepper(64, 3, 1, OR_TOWER_REFERENCE);
    bad |= stepper(64, 3, 1, OR_TOWER_CORRECT);
    bad |= stepper(64, 4, 2, OR_TOWER_REFERENCE);   /* W-cycle */
    printf(bad ? "FAIL\n" : "OK\n");
    return bad;
}
