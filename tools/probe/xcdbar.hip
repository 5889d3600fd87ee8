// xcdbar.hip -- what a barrier among the workgroups of ONE XCD costs against
// a kernel boundary (the fixed cost the small levels of a W-cycle pay ~1000
// times per cycle, DESIGN.md section 4 "W-cycles (round 5)").
//
// k_bar: a grid of 8*P workgroups of which only blockIdx % 8 == 0 work (the
// dispatcher deals workgroups round-robin over the 8 XCDs, so the P workers
// share XCD 0 and its L2); each of PH phases ends with an arrival on an
// agent-scope counter and a poll for all P arrivals.  Every poll is bounded
// (LIMIT polls, then the workgroup records a failure and leaves), so the
// grid always drains.  rel = 1 adds an agent-scope release fence before each
// arrival (the L2 write-back a cross-XCD hand-off would need).
// The boundary reference: PH back-to-back launches of an empty kernel.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/xcdbar tools/probe/xcdbar.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr long LIMIT = 1L << 22;

__global__ __launch_bounds__(1024) void k_bar(int *ctr, int P, int PH, int rel, int *fail,
                                              unsigned long long *t) {
    if (blockIdx.x % 8 != 0) return;
    const int w = blockIdx.x / 8;
    if (w >= P) return;
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    const unsigned long long t0 = wall_clock64();
    for (int p = 0; p < PH; ++p) {
        __syncthreads();
        if (threadIdx.x == 0 && !bad) {
            if (rel) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int want = P * (p + 1);
            long spins = 0;
            while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
                if (++spins > LIMIT) {
                    bad = 1;
                    break;
                }
            }
        }
        __syncthreads();
        if (bad) break;
    }
    if (threadIdx.x == 0) {
        if (bad) atomicAdd(fail, 1);
        if (w == 0) {
            t[0] = t0;
            t[1] = wall_clock64();
        }
    }
}

__global__ void k_empty(int *x) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && x[0] == 12345) x[1] = 1;
}

int main() {
    int dev = 0, khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    int *ctr, *fail;
    unsigned long long *t;
    CK(hipMalloc(&ctr, 64));
    CK(hipMalloc(&fail, 64));
    CK(hipMalloc(&t, 64));
    const int PH = 200;
    for (int rel = 0; rel < 2; ++rel)
        for (int P : {4, 8, 16, 32}) {
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipMemset(ctr, 0, 64));
                CK(hipMemset(fail, 0, 64));
                hipLaunchKernelGGL(k_bar, dim3(8 * P), dim3(1024), 0, 0, ctr, P, PH, rel, fail, t);
                CK(hipDeviceSynchronize());
                unsigned long long ht[2];
                int hf = 0;
                CK(hipMemcpy(ht, t, 16, hipMemcpyDeviceToHost));
                CK(hipMemcpy(&hf, fail, 4, hipMemcpyDeviceToHost));
                const double us = (double)(ht[1] - ht[0]) / (khz * 1e-3) / PH;
                if (rep == 2)
                    printf("{\"probe\": \"xcd_barrier\", \"release\": %d, \"workgroups\": %d, "
                           "\"us_per_phase\": %.3f, \"failed_workgroups\": %d}\n",
                           rel, P, us, hf);
            }
        }
    for (int G : {8, 64, 256}) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(a, 0));
            for (int p = 0; p < PH; ++p) hipLaunchKernelGGL(k_empty, dim3(G), dim3(1024), 0, 0, ctr);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep == 2)
                printf("{\"probe\": \"kernel_boundary\", \"workgroups\": %d, \"us_per_launch\": %.3f}\n",
                       G, ms * 1e3 / PH);
        }
    }
    return 0;
}
