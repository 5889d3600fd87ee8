// check_division.c -- the smoother's division (kernels.hip div_diag) is bitwise IEEE division.
//
// q0 = RN(a*y) with y = RN(1/d), r = fma(-q0, d, a) (exact), q = r == 0 ? q0 : fma(r, y, q0).
// Markstein's theorem says q = RN(a/d) when y = RN(1/d) and q0 is within one ulp; this
// program checks it on random numerators for every diagonal 1-4*rr*nu the solver uses
// (N = 8..65536, all levels, nu in {-4e-4, -0.01}) and on random divisors.
// usage: check_division [samples_per_divisor] [random_divisor_samples]
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static uint64_t s = 88172645463325252ull;
static inline uint64_t xr(void){ s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double rnd_double(void){ uint64_t b = xr(); // random finite normal double in moderate range
  uint64_t e = 1023 - 200 + (xr() % 400); b = (b & 0x800FFFFFFFFFFFFFull) | (e << 52); double d; memcpy(&d,&b,8); return d; }
int main(int argc, char **argv){
  long per = argc > 1 ? atol(argv[1]) : 20000000, rnd = argc > 2 ? atol(argv[2]) : 200000000;
  long bad = 0, tot = 0;
  double ds[64]; int nd = 0;
  // the actual divisors: dgs = 1 - 4*rr*nu for N up to 65536, all levels, nu in {-4e-4,-0.01}
  double nus[2] = {-4e-4, -0.01};
  for (int N = 8; N <= 65536; N *= 2) for (int q = 0; q < 2; q++) {
    double k = (1.0/N)/10; double h = 1.0/N;
    for (int l = 0; (N >> l) >= 2 && nd < 60; l++, h *= 2) { double rr = 0.5*k/(h*h); ds[nd++] = 1.0 - 4.0*rr*nus[q]; if (nd >= 60) break; }
  }
  for (int i = 0; i < nd; i++) {
    double d = ds[i], y = 1.0 / d;
    for (long t = 0; t < per; t++) {
      double a = rnd_double();
      double q0 = a * y; double r = fma(-q0, d, a); double qq = (r == 0.0) ? q0 : fma(r, y, q0);
      double ex = a / d; tot++;
      if (memcmp(&qq, &ex, 8)) { if (bad < 10) printf("MISMATCH d=%.17g a=%.17g got=%.17g exp=%.17g\n", d, a, qq, ex); bad++; }
    }
  }
  // random divisors too
  for (long t = 0; t < rnd; t++) {
    double d = rnd_double(); if (d < 0) d = -d; double y = 1.0/d; double a = rnd_double();
    double q0 = a * y; double r = fma(-q0, d, a); double qq = (r == 0.0) ? q0 : fma(r, y, q0);
    double ex = a / d; tot++;
    if (memcmp(&qq, &ex, 8)) { if (bad < 20) printf("MISMATCH2 d=%.17g a=%.17g got=%.17g exp=%.17g\n", d, a, qq, ex); bad++; }
  }
  printf("divisors %d, tests %ld, mismatches %ld\n", nd, tot, bad);
  return bad != 0;
}
