// Grid-barrier probe (experiment): the cost of one grid-wide barrier inside a
// persistent kernel (every workgroup resident) against the launch-to-launch
// time of back-to-back dependent small kernels.  Each phase every workgroup
// writes a row of a buffer and, after the barrier, reads a row another
// workgroup (on another XCD) wrote, so the barrier's release/acquire is
// exercised.  The spin has a wall-clock limit: a non-resident grid fails the
// check instead of hanging.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ bool grid_sync(unsigned *bar, unsigned target, int *err) {
    __syncthreads();
    __shared__ int bad;
    if (threadIdx.x == 0) {
        bad = 0;
        __threadfence();
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t0 = wall_clock64();
        while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > 20000000ull) {   // 200 ms at 100 MHz
                bad = 1;
                atomicExch(err, 1);
                break;
            }
        }
    }
    __syncthreads();
    return bad == 0;
}

__global__ __launch_bounds__(256) void k_persist(unsigned *bar, double *buf, int phases, int *err,
                                                 double *out) {
    const unsigned G = gridDim.x;
    double acc = 0;
    for (int p = 0; p < phases; ++p) {
        buf[(long)blockIdx.x * 256 + threadIdx.x] = p + threadIdx.x;
        if (!grid_sync(bar, (unsigned)(2 * p + 1) * G, err)) return;
        acc += buf[(long)((blockIdx.x + 13) % G) * 256 + threadIdx.x];
        // second barrier so the next phase's writes do not race the reads
        if (!grid_sync(bar, (unsigned)(2 * p + 2) * G, err)) return;
    }
    if (acc == -1.0) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_step(double *buf, int p) {
    const unsigned G = gridDim.x;
    double v = buf[(long)((blockIdx.x + 13) % G) * 256 + threadIdx.x];
    buf[(long)blockIdx.x * 256 + threadIdx.x] = v + p;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int per = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_persist, 256, 0);
    printf("CUs %d, resident 256-thread blocks per CU %d\n", cus, per);
    unsigned *bar;
    int *err;
    double *buf, *out;
    hipMalloc(&bar, 64);
    hipMalloc(&err, 64);
    hipMalloc(&buf, (size_t)4096 * 256 * 8);
    hipMalloc(&out, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int phases = 500;
    for (int G : {64, 256, 512, 1024}) {
        if (G > cus * per) continue;
        for (int rep = 0; rep < 2; ++rep) {
            hipMemset(bar, 0, 64);
            hipMemset(err, 0, 64);
            hipDeviceSynchronize();
            hipEventRecord(e0);
            k_persist<<<G, 256>>>(bar, buf, phases, err, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            int h = 0;
            hipMemcpy(&h, err, 4, hipMemcpyDeviceToHost);
            printf("persistent G=%d: %.2f us per barrier%s\n", G, ms * 1e3 / (2 * phases),
                   h ? "  (TIMED OUT)" : "");
            if (h) return 1;
        }
    }
    for (int G : {64, 256, 1024}) {
        for (int rep = 0; rep < 2; ++rep) {
            hipDeviceSynchronize();
            hipEventRecord(e0);
            for (int p = 0; p < 2 * phases; ++p) k_step<<<G, 256>>>(buf, p);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("launches G=%d: %.2f us per dependent launch\n", G, ms * 1e3 / (2 * phases));
        }
    }
    return 0;
}
