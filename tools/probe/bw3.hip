// Row-pitch sweep for the column-strip march (experiment): does the row pitch
// (partition camping across HBM channels) set the march's bandwidth?
//   march: wave = one 1-KiB column strip, P = 4 rows of loads in flight,
//   4 in / 1 out, static segments (one per wave), 8 waves per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int P>
__global__ __launch_bounds__(256) void k_march(const double2 *__restrict__ a,
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
        ra[p] = a[off]; rb[p] = b[off]; rc[p] = c[off]; rd[p] = d[off];
    }
    for (int r = r0; r < r1; r += P) {
#pragma unroll
        for (int p = 0; p < P; ++p) {
            double2 v = ra[p];
            v.x += rb[p].x + rc[p].x + rd[p].x;
            v.y += rb[p].y + rc[p].y + rd[p].y;
            if (r + p < r1) o[(long)(r + p) * pitch2 + col] = v;
            const long off = (long)min(r + p + P, r1 - 1) * pitch2 + col;
            ra[p] = a[off]; rb[p] = b[off]; rc[p] = c[off]; rd[p] = d[off];
        }
    }
}

int main() {
    const long bytes = 2L << 30;
    double2 *buf[5];
    for (auto &p : buf) {
        if (hipMalloc(&p, bytes + (64 << 20)) != hipSuccess) return 1;
        (void)hipMemset(p, 0, bytes);
    }
    int cus;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int strips = 128;   // 128 x 1 KiB = 16384 doubles per row (N=16384 level 0)
    // pad in bytes beyond 128 KiB
    for (long pad : {0L, 64L, 128L, 256L, 384L, 512L, 640L, 1024L, 1152L, 2048L, 3072L, 4096L,
                     4224L, 8192L, 8320L}) {
        const long pitch2 = (131072 + pad) / 16;
        const int rows = (int)(bytes / 16 / pitch2) - 1;
        const double mb = 5.0 * rows * strips * 1024.0;
        for (int wpc : {8}) {
            const long waves = (long)cus * wpc;
            const int segs = (int)(waves / strips);
            const unsigned g = (unsigned)(((long)segs * strips + 3) / 4);
            auto go = [&] {
                k_march<4><<<g, 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], pitch2, rows,
                                       strips, segs);
            };
            go();
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) go();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            printf("pitch 128KiB+%5ld B: %.0f GB/s\n", pad, mb * 5 / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
