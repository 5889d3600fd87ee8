// coarse_phases.hip -- where the coarsest solve's ~10 us go (DESIGN.md
// section 4 "W-cycles (round 5)"): stencil.h coarse_lds_body timed from inside
// one 1024-thread workgroup with wall_clock64 (thread 0, after a barrier), at
// maxit 0 (set-up loads + store only), 1 iteration, and reps 2, on a 64 x 64
// coarsest level whose fields were just written by another kernel (cold L2,
// as in a V-cycle) or re-read (warm).
//   hipcc --offload-arch=gfx950 -O3 -I hpcclassmultigridproject_amd/csrc \
//         -o tools/probe/coarse_phases tools/probe/coarse_phases.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "stencil.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace mgx;

__global__ __launch_bounds__(1024) void k_probe(double *u, const double *rhs, const double *v1,
                                                const double *v2, int n, long pitch, Coef c,
                                                int maxit, int reps, double *stats,
                                                unsigned long long *t) {
    __shared__ double su[kCoarseLdsNP * kCoarseLdsNP];
    __shared__ double lds[16];
    __shared__ double s_norm;
    __syncthreads();
    const unsigned long long t0 = wall_clock64();
    coarse_lds_body<true>(su, lds, &s_norm, u, rhs, v1, v2, n, pitch, c, 1e-30, maxit, 1, reps,
                          stats, true);
    __syncthreads();
    if (threadIdx.x == 0) {
        t[0] = t0;
        t[1] = wall_clock64();
    }
}

__global__ void k_touch(double *a, long cnt) {   // rewrite the fields (cold L2 for the probe)
    for (long i = blockIdx.x * 256L + threadIdx.x; i < cnt; i += 256L * gridDim.x) a[i] = a[i] + 0.0;
}

int main() {
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    const int n = 64;
    const long pitch = 80, cnt = (n + 1) * pitch;
    std::vector<double> h(cnt);
    for (long i = 0; i < cnt; ++i) h[i] = 1e-3 * (double)((i * 7919) % 1000) - 0.5;
    double *u, *rhs, *v1, *v2, *stats;
    unsigned long long *t;
    for (double **p : {&u, &rhs, &v1, &v2}) {
        CK(hipMalloc(p, cnt * sizeof(double)));
        CK(hipMemcpy(*p, h.data(), cnt * sizeof(double), hipMemcpyHostToDevice));
    }
    CK(hipMalloc(&stats, 64));
    CK(hipMalloc(&t, 64));
    Coef c{};   // kernels.hip make_coef for k = dt, nu, h = 1/64, fp_mode fma
    {
        const double k = 1.0 / 16384 / 10, nu = -4e-4, hh = 1.0 / 64;
        c.rr = 0.5 * k / (hh * hh);
        c.nu = nu;
        c.h = hh;
        c.dgs = 1.0 - 4.0 * c.rr * nu;
        c.drhs = 1.0 + 4.0 * c.rr * nu;
        c.rdgs = 1.0 / c.dgs;
        c.dsign = 0u;
        c.g = c.rr / c.dgs;
        c.gn = c.g * nu;
        c.c2 = -2.0 * c.gn;
        c.fm = 1;
    }
    struct Case { const char *name; int maxit, reps, cold; };
    for (Case k : {Case{"setup+store", 0, 1, 1}, Case{"1 iteration", 1, 1, 1},
                   Case{"2 reps x 1 iteration", 1, 2, 1}, Case{"4 iterations", 4, 1, 1},
                   Case{"1 iteration, warm", 1, 1, 0}}) {
        double best = 1e30;
        for (int rep = 0; rep < 20; ++rep) {
            if (k.cold)
                for (double *p : {rhs, v1, v2}) hipLaunchKernelGGL(k_touch, dim3(8), dim3(256), 0, 0, p, cnt);
            hipLaunchKernelGGL(k_probe, dim3(1), dim3(1024), 0, 0, u, rhs, v1, v2, n, pitch, c,
                               k.maxit, k.reps, stats, t);
            CK(hipDeviceSynchronize());
            unsigned long long ht[2];
            CK(hipMemcpy(ht, t, 16, hipMemcpyDeviceToHost));
            const double us = (double)(ht[1] - ht[0]) / (khz * 1e-3);
            if (rep >= 2 && us < best) best = us;
        }
        printf("{\"probe\": \"coarse_phases\", \"case\": \"%s\", \"us_in_kernel_min\": %.3f}\n",
               k.name, best);
    }
    return 0;
}
