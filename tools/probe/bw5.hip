// Streaming-bandwidth probe, round 6 (experiment, not product): does a
// column-strip row march read faster when its rows are prefetched by LDS-DMA
// (global_load_lds_dwordx4 into a wave-private LDS ring, no VGPR cost, so the
// ring can be deeper) than with the register prefetch of bw2.hip's k_march?
// Same shape as bw2: 4 inputs + 1 output, 1-KiB strips of a 16384+128-double
// pitched array, one wave per (strip, row segment).
//   rmarch<P>  : register prefetch, P rows ahead (bw2's k_march)
//   lmarch<D>  : LDS ring of D rows x 4 arrays x 1 KiB per wave, counted
//                s_waitcnt vmcnt before reading the oldest row back
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((address_space(3))) void lds_void;

template <int P>
__global__ __launch_bounds__(256) void k_rmarch(const double2 *__restrict__ a,
                                                const double2 *__restrict__ b,
                                                const double2 *__restrict__ c,
                                                const double2 *__restrict__ d,
                                                double2 *__restrict__ o, long pitch2, int rows,
                                                int strips, int segs) {
    const int l = threadIdx.x & 63;
    const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int strip = (int)(wave % strips);
    const int seg = (int)(wave / strips);
    if (seg >= segs) return;
    const int r0 = (int)((long)rows * seg / segs), r1 = (int)((long)rows * (seg + 1) / segs);
    const long col = (long)strip * 64 + l;
    double2 ra[P], rb[P], rc[P], rd[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const long off = (long)min(r0 + p, r1 - 1) * pitch2 + col;
        ra[p] = a[off];
        rb[p] = b[off];
        rc[p] = c[off];
        rd[p] = d[off];
    }
    for (int r = r0; r < r1; r += P) {
#pragma unroll
        for (int p = 0; p < P; ++p) {
            double2 v = ra[p];
            v.x += rb[p].x + rc[p].x + rd[p].x;
            v.y += rb[p].y + rc[p].y + rd[p].y;
            if (r + p < r1) o[(long)(r + p) * pitch2 + col] = v;
            const long off = (long)min(r + p + P, r1 - 1) * pitch2 + col;
            ra[p] = a[off];
            rb[p] = b[off];
            rc[p] = c[off];
            rd[p] = d[off];
        }
    }
}

// imarch: the rmarch march over a band-interleaved row layout -- band b's
// k-th row lives at physical row k * segs + b, so the rows the bands march at
// one moment are adjacent in memory (one compact window, like a flat stream)
template <int P, bool IL>
__global__ __launch_bounds__(256) void k_imarch(const double2 *__restrict__ a,
                                                const double2 *__restrict__ b,
                                                const double2 *__restrict__ c,
                                                const double2 *__restrict__ d,
                                                double2 *__restrict__ o, long pitch2, int R,
                                                int strips, int segs) {
    const int l = threadIdx.x & 63;
    const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int strip = (int)(wave % strips);
    const int seg = (int)(wave / strips);
    if (seg >= segs) return;
    const long col = (long)strip * 64 + l;
    const long step = IL ? (long)segs * pitch2 : pitch2;
    const long base = (IL ? (long)seg : (long)seg * R) * pitch2 + col;
    double2 ra[P], rb[P], rc[P], rd[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const long off = base + (long)p * step;
        ra[p] = a[off];
        rb[p] = b[off];
        rc[p] = c[off];
        rd[p] = d[off];
    }
    for (int k = 0; k < R; k += P) {
#pragma unroll
        for (int p = 0; p < P; ++p) {
            double2 v = ra[p];
            v.x += rb[p].x + rc[p].x + rd[p].x;
            v.y += rb[p].y + rc[p].y + rd[p].y;
            if (k + p < R) o[base + (long)(k + p) * step] = v;
            const long off = base + (long)min(k + p + P, R - 1) * step;
            ra[p] = a[off];
            rb[p] = b[off];
            rc[p] = c[off];
            rd[p] = d[off];
        }
    }
}

__device__ __forceinline__ double2 lds_read16(unsigned addr) {
    double2 v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    // gfx9 s_waitcnt: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14]
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

template <int D>
__device__ __forceinline__ void issue_row(const double2 *a, const double2 *b, const double2 *c,
                                          const double2 *d, long off, char *ring, int slot) {
    char *s = ring + slot * 4096;
    __builtin_amdgcn_global_load_lds((const void *)(a + off), (lds_void *)(s), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void *)(b + off), (lds_void *)(s + 1024), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void *)(c + off), (lds_void *)(s + 2048), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void *)(d + off), (lds_void *)(s + 3072), 16, 0, 0);
}

template <int D>
__global__ __launch_bounds__(256) void k_lmarch(const double2 *__restrict__ a,
                                                const double2 *__restrict__ b,
                                                const double2 *__restrict__ c,
                                                const double2 *__restrict__ d,
                                                double2 *__restrict__ o, long pitch2, int rows,
                                                int strips, int segs) {
    extern __shared__ char smem[];
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long wave = (long)blockIdx.x * 4 + w;
    const int strip = (int)(wave % strips);
    const int seg = (int)(wave / strips);
    if (seg >= segs) return;
    const int r0 = (int)((long)rows * seg / segs), r1 = (int)((long)rows * (seg + 1) / segs);
    const long col = (long)strip * 64 + l;
    char *ring = smem + w * D * 4096;
    const unsigned ring_addr = (unsigned)(size_t)(lds_void *)ring + l * 16;
#pragma unroll
    for (int p = 0; p < D; ++p) issue_row<D>(a, b, c, d, (long)min(r0 + p, r1 - 1) * pitch2 + col,
                                             ring, p);
    int slot = 0;
    for (int r = r0; r < r1; ++r) {
        // the oldest row's 4 loads have retired once at most 4 (D - 1) loads
        // (and the stores issued since, counted conservatively) remain
        wait_vm<4 * (D - 1)>();
        const unsigned base = ring_addr + slot * 4096;
        const double2 va = lds_read16(base), vb = lds_read16(base + 1024),
                      vc = lds_read16(base + 2048), vd = lds_read16(base + 3072);
        issue_row<D>(a, b, c, d, (long)min(r + D, r1 - 1) * pitch2 + col, ring, slot);
        double2 v = va;
        v.x += vb.x + vc.x + vd.x;
        v.y += vb.y + vc.y + vd.y;
        o[(long)r * pitch2 + col] = v;
        slot = slot + 1 == D ? 0 : slot + 1;
    }
    wait_vm<0>();
}

__global__ void k_fill(double2 *p, long n, double s) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        p[i] = make_double2(s * (double)(i & 1023), s + (double)(i % 7));
}

__global__ void k_check(const double2 *o, long pitch2, int rows, double *err) {
    // o = a + b + c + d with a..d from k_fill(s = 1, 2, 3, 4)
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < (long)rows * pitch2;
         i += (long)gridDim.x * blockDim.x) {
        const double x = 10.0 * (double)(i & 1023), y = 10.0 + 4.0 * (double)(i % 7);
        const double e = fabs(o[i].x - x) + fabs(o[i].y - y);
        if (e != 0.0) atomicAdd(err, e);
    }
}

static hipEvent_t e0, e1;
template <typename F>
static double timeit(F go, double bytes) {
    go();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) go();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return bytes * 5 / (ms * 1e-3) / 1e9;
}

int main() {
    const long bytes = 2L << 30;
    const long n = bytes / 16;
    double2 *buf[5];
    for (int i = 0; i < 5; ++i) {
        if (hipMalloc(&buf[i], bytes) != hipSuccess) return 1;
        k_fill<<<4096, 256>>>(buf[i], n, (double)(i + 1));
    }
    double *err;
    hipMalloc(&err, 8);
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int cus;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    auto A = buf[0], B = buf[1], Cc = buf[2], D = buf[3], O = buf[4];
    const long pitch2 = 8256;
    const int rows = (int)(n / pitch2);
    const int strips = (int)(pitch2 / 64);
    const double mbytes = 5.0 * rows * pitch2 * 16;
    auto check = [&](const char *what) {
        hipMemset(err, 0, 8);
        k_check<<<4096, 256>>>(O, pitch2, rows, err);
        double h;
        hipMemcpy(&h, err, 8, hipMemcpyDeviceToHost);
        if (h != 0.0) printf("  !! %s wrong: err %g\n", what, h);
        hipMemset(O, 0, bytes);
    };
    hipFuncSetAttribute((const void *)k_lmarch<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void *)k_lmarch<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void *)k_lmarch<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int wpc : {8, 16}) {
        const long waves = (long)cus * wpc;
        const int segs = (int)(waves / strips);
        const unsigned g = (unsigned)(((long)segs * strips + 3) / 4);
        printf("rmarch P=2 waves/CU~%d: %.0f GB/s\n", wpc, timeit([&] {
                   k_rmarch<2><<<g, 256>>>(A, B, Cc, D, O, pitch2, rows, strips, segs);
               }, mbytes));
        check("rmarch2");
        printf("rmarch P=4 waves/CU~%d: %.0f GB/s\n", wpc, timeit([&] {
                   k_rmarch<4><<<g, 256>>>(A, B, Cc, D, O, pitch2, rows, strips, segs);
               }, mbytes));
        check("rmarch4");
    }
    for (int wpc : {8, 16}) {
        const long waves = (long)cus * wpc;
        const int segs = (int)(waves / strips);
        const int R = rows / segs;
        const unsigned g = (unsigned)(((long)segs * strips + 3) / 4);
        const double ib = 5.0 * (double)R * segs * pitch2 * 16;
        printf("imarch contiguous P=2 waves/CU~%d bands %d: %.0f GB/s\n", wpc, segs, timeit([&] {
                   k_imarch<2, false><<<g, 256>>>(A, B, Cc, D, O, pitch2, R, strips, segs);
               }, ib));
        printf("imarch interleaved P=2 waves/CU~%d bands %d: %.0f GB/s\n", wpc, segs, timeit([&] {
                   k_imarch<2, true><<<g, 256>>>(A, B, Cc, D, O, pitch2, R, strips, segs);
               }, ib));
        printf("imarch interleaved P=4 waves/CU~%d bands %d: %.0f GB/s\n", wpc, segs, timeit([&] {
                   k_imarch<4, true><<<g, 256>>>(A, B, Cc, D, O, pitch2, R, strips, segs);
               }, ib));
    }
    // LDS per workgroup = 4 waves x D x 4 KiB; waves per CU limited by 160 KiB
    for (int wpc : {4, 8, 16}) {
        const long waves = (long)cus * wpc;
        const int segs = (int)(waves / strips);
        const unsigned g = (unsigned)(((long)segs * strips + 3) / 4);
        if (wpc * 2 * 4096 <= 160 * 1024) {
            printf("lmarch D=2 waves/CU~%d: %.0f GB/s\n", wpc, timeit([&] {
                       k_lmarch<2><<<g, 256, 4 * 2 * 4096>>>(A, B, Cc, D, O, pitch2, rows, strips,
                                                            segs);
                   }, mbytes));
            check("lmarch2");
        }
        if (wpc * 4 * 4096 <= 160 * 1024) {
            printf("lmarch D=4 waves/CU~%d: %.0f GB/s\n", wpc, timeit([&] {
                       k_lmarch<4><<<g, 256, 4 * 4 * 4096>>>(A, B, Cc, D, O, pitch2, rows, strips,
                                                            segs);
                   }, mbytes));
            check("lmarch4");
        }
        if (wpc * 8 * 4096 <= 160 * 1024) {
            printf("lmarch D=8 waves/CU~%d: %.0f GB/s\n", wpc, timeit([&] {
                       k_lmarch<8><<<g, 256, 4 * 8 * 4096>>>(A, B, Cc, D, O, pitch2, rows, strips,
                                                            segs);
                   }, mbytes));
            check("lmarch8");
        }
    }
    return 0;
}
