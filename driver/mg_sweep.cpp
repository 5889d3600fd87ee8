// driver/mg_sweep.cpp -- N-sweep timing harness, the GPU
// counterpart of the reference's mg_timer.cu:212-268 and of the OMP harness
// multigrid_strongsc.cpp:251-262.
//
// For N = Nmin, 2Nmin, ..., Nmax (maxlvl = log2(N)-4 unless -L is given):
//   * the 100-step time stepper on the GPU (context create + upload + steps +
//     download, as mg_timer.cu times it), printed as
//     "Time elapsed for grid size %d: %g ms" and appended to <prefix>cudatime.txt
//     as "%d\t%f\n" (N, seconds) -- the format speedupplot.py reads;
//   * V-cycle throughput: `cycles` fixed V-cycles (+ residual norm) after one
//     warm-up, (N-1)^2 * cycles / s, appended to <prefix>gpups.txt as
//     "%d\t%e\n" (N, grid-point-updates/s).
// Flags: -Nmin n -Nmax n -L maxlvl -steps s -cycles c -out prefix
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "mgx.h"

static void die(int rc, const char *what) {
    if (rc != MGX_OK && rc != MGX_E_NOCONV) {
        fprintf(stderr, "%s failed (%d): %s\n", what, rc, mgx_last_error());
        exit(1);
    }
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

int main(int argc, char **argv) {
    long nmin = 32, nmax = 4096;
    int fixed_L = -1, steps = 100, cycles = 10;
    std::string prefix;
    for (int a = 1; a < argc; ++a) {
        std::string k = argv[a];
        if (a + 1 >= argc) {
            fprintf(stderr, "missing value for %s\n", k.c_str());
            return 2;
        }
        const char *v = argv[++a];
        if (k == "-Nmin") nmin = atol(v);
        else if (k == "-Nmax") nmax = atol(v);
        else if (k == "-L") fixed_L = atoi(v);
        else if (k == "-steps") steps = atoi(v);
        else if (k == "-cycles") cycles = atoi(v);
        else if (k == "-out") prefix = v;
        else {
            fprintf(stderr, "unknown flag %s\n", k.c_str());
            return 2;
        }
    }
    FILE *ft = fopen((prefix + "cudatime.txt").c_str(), "w");
    FILE *fg = fopen((prefix + "gpups.txt").c_str(), "w");
    if (!ft || !fg) {
        perror("output file");
        return 1;
    }
    for (long N = nmin; N <= nmax; N <<= 1) {
        const int maxlvl = fixed_L > 0 ? fixed_L : std::max(1, int(log2(N)) - 4);
        const double dx = 1.0 / N, dt = dx / 10, T = steps * dt, nu = -4 * 1e-4, tol = 1e-6;
        const size_t cnt = (size_t)(N + 1) * (N + 1);
        std::vector<double> u0(cnt), v1(cnt), v2(cnt), uT(cnt);
        die(mgx_init_problem(u0.data(), v1.data(), v2.data(), N, 0), "init_problem");

        // time stepper, timed like mg_timer.cu (device setup + steps + copy back)
        double t0 = now();
        die(mgx_timestepper(uT.data(), u0.data(), v1.data(), v2.data(), nu, maxlvl, N, dt, T,
                            dx, tol, 1),
            "mgx_timestepper");
        const double secs = now() - t0;
        printf("Time elapsed for grid size %ld: %g ms\n", N, secs * 1e3);
        fprintf(ft, "%ld\t%f\n", N, secs);

        // fixed-count V-cycles on a resident context
        mgx_ctx *ctx = nullptr;
        die(mgx_create(&ctx, N, maxlvl, dt, nu, nullptr), "mgx_create");
        die(mgx_upload(ctx, u0.data(), v1.data(), v2.data()), "mgx_upload");
        die(mgx_rhs(ctx), "mgx_rhs");
        double r = 0;
        die(mgx_run_cycles(ctx, 1, &r), "warm-up");
        die(mgx_synchronize(ctx), "sync");
        t0 = now();
        die(mgx_run_cycles(ctx, cycles, &r), "run_cycles");
        die(mgx_synchronize(ctx), "sync");
        const double vs = now() - t0;
        const double gpups = double(N - 1) * double(N - 1) * cycles / vs;
        printf("  V-cycle (L=%d): %.4f ms, %.3e grid-point-updates/s\n", maxlvl,
               vs / cycles * 1e3, gpups);
        fprintf(fg, "%ld\t%e\n", N, gpups);
        mgx_destroy(ctx);
    }
    fclose(ft);
    fclose(fg);
    return 0;
}
