// Access-pattern probe for the column-strip march (experiment, not product):
// is the ~5.2 TB/s ceiling of a 4-in/1-out row march set by the
// four input fields living 2 GiB apart, or by how many contiguous bytes a
// workgroup touches per row?
//   sep   : 5 separate fields (as the solver: u, rhs, v1, v2 in, u out)
//   ilv   : one buffer, the 5 fields' rows interleaved (row r of field k at
//           (5 r + k) * pitch): a workgroup's loads of one step share pages
//   wide W: separate fields, W waves per workgroup on W adjacent strips
//           (W KiB contiguous per row and field), same waves per CU
//   flat  : the same bytes as a flat 4-in/1-out stream (one 16-B element per
//           lane, one workgroup per 4 KiB), the measured stream ceiling
// hipcc --offload-arch=gfx950 -O3 -o /tmp/bw4 tools/probe/bw4.hip && /tmp/bw4
#include <hip/hip_runtime.h>
#include <cstdio>

template <int P>
__global__ void k_march(const double2 *__restrict__ a, const double2 *__restrict__ b,
                        const double2 *__restrict__ c, const double2 *__restrict__ d,
                        double2 *__restrict__ o, long pitch2, int rows, int strips, int segs,
                        int wpb) {
    const int l = threadIdx.x & 63;
    const long wave = (long)blockIdx.x * wpb + (threadIdx.x >> 6);
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

__global__ __launch_bounds__(256) void k_flat(const double2 *__restrict__ a,
                                              const double2 *__restrict__ b,
                                              const double2 *__restrict__ c,
                                              const double2 *__restrict__ d,
                                              double2 *__restrict__ o, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double2 v = a[i];
    const double2 x = b[i], y = c[i], z = d[i];
    v.x += x.x + y.x + z.x;
    v.y += x.y + y.y + z.y;
    __builtin_nontemporal_store(v.x, &o[i].x);
    __builtin_nontemporal_store(v.y, &o[i].y);
}

int main() {
    const long row_b = 131072;                 // 16384 doubles (N=16384 level 0)
    const long pitch2 = row_b / 16;
    const int rows = 16384;
    const long bytes = row_b * rows;           // 2 GiB per field
    const int strips = 128;
    double2 *sep[5], *ilv, *stg[5];
    for (auto &p : sep)
        if (hipMalloc(&p, bytes) != hipSuccess || hipMemset(p, 0, bytes) != hipSuccess) return 1;
    for (auto &p : stg)
        if (hipMalloc(&p, bytes + (1 << 20)) != hipSuccess ||
            hipMemset(p, 0, bytes + (1 << 20)) != hipSuccess)
            return 1;
    if (hipMalloc(&ilv, 5 * bytes) != hipSuccess || hipMemset(ilv, 0, 5 * bytes) != hipSuccess)
        return 1;
    int cus;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double moved = 5.0 * bytes;
    auto timeit = [&](const char *name, auto go) {
        go();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) go();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s %6.0f GB/s\n", name, moved * 5 / (ms * 1e-3) / 1e9);
    };
    const long waves = (long)cus * 8;          // 8 waves per CU, as the solver
    const int segs = (int)(waves / strips);
    for (int rep = 0; rep < 2; ++rep) {
        if (rep) printf("--\n");
        for (int wpb : {4, 8, 16}) {
            const unsigned g = (unsigned)(((long)segs * strips + wpb - 1) / wpb);
            char nm[64];
            snprintf(nm, sizeof nm, "sep  march, %2d waves/WG", wpb);
            timeit(nm, [&] {
                k_march<4><<<g, 64 * wpb>>>(sep[0], sep[1], sep[2], sep[3], sep[4], pitch2, rows,
                                            strips, segs, wpb);
            });
            snprintf(nm, sizeof nm, "ilv  march, %2d waves/WG", wpb);
            timeit(nm, [&] {
                k_march<4><<<g, 64 * wpb>>>(ilv, ilv + pitch2, ilv + 2 * pitch2, ilv + 3 * pitch2,
                                            ilv + 4 * pitch2, 5 * pitch2, rows, strips, segs,
                                            wpb);
            });
        }
        // separate fields whose bases are staggered by k * st bytes (the
        // 2 MiB-aligned allocations otherwise put the same column of every
        // field on the same channel)
        for (long st : {256L, 1024L, 2048L, 4096L, 8192L, 16384L, 65536L, 135168L}) {
            const unsigned g = (unsigned)(((long)segs * strips + 3) / 4);
            char nm[64];
            snprintf(nm, sizeof nm, "sep  march, stagger %6ld B", st);
            timeit(nm, [&] {
                k_march<4><<<g, 256>>>(stg[0], stg[1] + st / 16, stg[2] + 2 * st / 16,
                                       stg[3] + 3 * st / 16, stg[4] + 4 * st / 16, pitch2, rows,
                                       strips, segs, 4);
            });
        }
        const long n = bytes / 16;
        timeit("flat stream (nt stores)", [&] {
            k_flat<<<(unsigned)((n + 255) / 256), 256>>>(sep[0], sep[1], sep[2], sep[3], sep[4],
                                                          n);
        });
    }
    return 0;
}
