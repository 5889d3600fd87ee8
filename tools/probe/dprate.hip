// fp64 VALU issue-rate probe (experiment): independent v_mul_f64 / v_add_f64 /
// v_fma_f64 chains, 8 per lane, WPC waves per CU.  Prints wave-instructions
// per SIMD per cycle-equivalent: cycles/instr at the measured clock.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int OP>
__global__ __launch_bounds__(256) void k(double *out, double a, double b, int iters) {
    double x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3 + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (OP == 0) x[i] = x[i] * a;
                else if (OP == 1) x[i] = x[i] + b;
                else x[i] = __builtin_fma(x[i], a, b);
            }
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
    if (s == 12345.678) out[threadIdx.x] = s;
}
int main() {
    double *o;
    hipMalloc(&o, 4096);
    int cus;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4096;
    for (int op = 0; op < 3; ++op)
        for (int wpc : {4, 8, 16}) {
            const int grid = cus * wpc / 4;
            auto go = [&] {
                if (op == 0) k<0><<<grid, 256>>>(o, 0.999999, 1e-9, iters);
                if (op == 1) k<1><<<grid, 256>>>(o, 0.999999, 1e-9, iters);
                if (op == 2) k<2><<<grid, 256>>>(o, 0.999999, 1e-9, iters);
            };
            go();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            go();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double winstr = (double)grid * 4 * iters * 128;   // wave-instructions
            const double per_simd = winstr / (cus * 4);
            printf("op=%d waves/CU=%d: %.3f ms, %.1f Gwave-instr/s per SIMD -> %.2f ns/instr, "
                   "%.1f TFLOP-ops/s chip (lanes)\n", op, wpc, ms, per_simd / (ms * 1e-3) / 1e9,
                   ms * 1e6 / per_simd, winstr * 64 / (ms * 1e-3) / 1e12);
        }
    return 0;
}
