// Streaming-bandwidth variants (experiment): copy / 4-in-1-out, unroll, nt.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef double d2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ double2 nt_ld(const double2 *p) {
    d2v v = __builtin_nontemporal_load((const d2v *)p);
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ void nt_st(double2 r, double2 *p) {
    d2v v = {r.x, r.y};
    __builtin_nontemporal_store(v, (d2v *)p);
}
template <int NIN, int U, bool NT>
__global__ __launch_bounds__(256) void k(const double2 *__restrict__ a, const double2 *__restrict__ b,
                                         const double2 *__restrict__ c, const double2 *__restrict__ d,
                                         double2 *__restrict__ o, long n) {
    const long stride = (long)gridDim.x * blockDim.x;
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        double2 v[U], y[U], z[U], w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long j = i + u * stride;
            if (NT) {
                v[u] = nt_ld(a + j);
                if (NIN > 1) { y[u] = nt_ld(b + j); z[u] = nt_ld(c + j); w[u] = nt_ld(d + j); }
            } else {
                v[u] = a[j];
                if (NIN > 1) { y[u] = b[j]; z[u] = c[j]; w[u] = d[j]; }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            double2 r = v[u];
            if (NIN > 1) { r.x += y[u].x + z[u].x + w[u].x; r.y += y[u].y + z[u].y + w[u].y; }
            if (NT) nt_st(r, o + i + u * stride);
            else o[i + u * stride] = r;
        }
    }
}

template <int NIN, int U, bool NT>
void run(double2 **buf, long n, int wgs_per_cu, int cus) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int grid = cus * wgs_per_cu;
    auto go = [&] { k<NIN, U, NT><<<grid, 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], n); };
    go();
    hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) go();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("nin=%d U=%d NT=%d wgs/cu=%d: %.1f GB/s\n", NIN, U, NT, wgs_per_cu,
           16.0 * n * (NIN + 1) * 10 / (ms * 1e-3) / 1e9);
}

int main() {
    const long n = (1L << 30) / 16;
    double2 *buf[5];
    for (auto &b : buf) { hipMalloc(&b, n * 16); hipMemset(b, 0, n * 16); }
    int cus; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int w : {4, 8, 16}) {
        run<1, 1, false>(buf, n, w, cus); run<1, 4, false>(buf, n, w, cus); run<1, 4, true>(buf, n, w, cus);
        run<4, 1, false>(buf, n, w, cus); run<4, 2, false>(buf, n, w, cus); run<4, 2, true>(buf, n, w, cus);
        run<4, 4, false>(buf, n, w, cus);
    }
    return 0;
}
