// driver/multigrid.cpp -- drop-in for the reference's ./multigrid (multigrid.cpp:188-293).
//
// Same defaults (N=256, maxlvl=log2(N)-4, nu=-4e-4, dt=dx/10, T=100dt, tol=1e-6,
// V-cycle), same output files (uT.txt and uTomp.txt, "%d\t%d\t%f\n", i outer,
// j inner; uTplot.py reads both) and the same stdout lines.  The solver
// control flow keeps the reference's shape -- multigrid() (mg_outer,
// :97-120) drives vcycle() (mg_inner, :17-92) which drives gs() -- but every
// op is a call through the C ABI of include/mgx.h (HIP kernels on the GPU).
//
// Run 1 ("reference" line) uses this driver-side control flow on top of the
// op-level entry points; run 2 ("fast path") is the library's own
// mgx_timestepper.  Both must agree bitwise; the printed error is their L1
// difference, as multigrid.cpp:261-266 prints serial vs OMP.
//
// Flags (all optional): -N n  -L maxlvl  -nu nu  -steps s  -tol t  -shape 1|2
//                       -nsmooth k  -tower 0|1  -out prefix  -cuda (also write uTcuda.txt)
//                       -fp bitwise|fma (run 2's arithmetic, mgx_options.fp_mode;
//                       fma: the printed error is then the fma path's L1 distance
//                       from the bitwise one)
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mgx.h"

static void die(int rc, const char *what) {
    if (rc != MGX_OK && rc != MGX_E_NOCONV) {
        fprintf(stderr, "%s failed (%d): %s\n", what, rc, mgx_last_error());
        exit(1);
    }
}

// gauss_seidel x sweeps on one level (multigrid.cpp:69-72)
static void gs(mgx_ctx *ctx, int level, int sweeps) { die(mgx_gs(ctx, level, sweeps), "gs"); }

// mg_inner (multigrid.cpp:17-92) expressed with the op-level entry points.
static void vcycle(mgx_ctx *ctx, int lvl, int maxlvl, int shape, int nsmooth) {
    for (int sh = 0; sh < shape; ++sh) {
        if (lvl == maxlvl - 1) {
            double res = 1.0;
            int i = 0;
            while (i < 1000 && res > 1e-5) {   // multigrid.cpp:60
                gs(ctx, lvl, 1);
                die(mgx_residual_norm(ctx, lvl, &res), "residual_norm");
                ++i;
            }
        } else {
            gs(ctx, lvl, nsmooth);
            die(mgx_restrict(ctx, lvl), "restrict");   // residual, restriction, u[l+1]=0
            vcycle(ctx, lvl + 1, maxlvl, shape, nsmooth);
            die(mgx_prolong_add(ctx, lvl), "prolong_add");
            gs(ctx, lvl, nsmooth);
        }
    }
}

// mg_outer (multigrid.cpp:97-120)
static int multigrid(mgx_ctx *ctx, int maxlvl, int shape, int nsmooth, double tol) {
    const int MAX_CYCLE = 50;
    double res0 = 0, res = 0;
    die(mgx_residual_norm(ctx, 0, &res0), "residual_norm");
    res = res0;
    int iter;
    for (iter = 0; iter < MAX_CYCLE && res / res0 > tol; iter++) {
        vcycle(ctx, 0, maxlvl, shape, nsmooth);
        die(mgx_residual_norm(ctx, 0, &res), "residual_norm");
    }
    if (iter == MAX_CYCLE) printf("multigrid did not converge in %d cycles\n", MAX_CYCLE);
    return iter;
}

// timestepper (multigrid.cpp:124-186) on a device-resident context
static void timestepper(double *uT, const double *u0, const double *v1, const double *v2,
                        double nu, int maxlvl, long n, double dt, double T, double tol,
                        int shape, int nsmooth, int tower) {
    mgx_options o;
    mgx_default_options(&o);
    o.shape = shape;
    o.nsmooth = nsmooth;
    o.tower_mode = tower;
    mgx_ctx *ctx = nullptr;
    die(mgx_create(&ctx, n, maxlvl, dt, nu, &o), "mgx_create");
    die(mgx_upload(ctx, u0, v1, v2), "mgx_upload");
    for (int it = 0; it < (int)(T / dt); it++) {
        die(mgx_rhs(ctx), "compute_rhs");
        multigrid(ctx, maxlvl, shape, nsmooth, tol);
    }
    die(mgx_download(ctx, uT), "mgx_download");
    mgx_destroy(ctx);
}

// multigrid.cpp:269-284's writer ("%d\t%d\t%f\n", i outer, j inner), formatted
// on all host threads by the library (mgx_write_uT; row blocks append)
static void write_uT(const char *path, const double *u, long N) {
    die(mgx_write_uT(path, u, N, 0, N + 1, 0, 0), path);
}

int main(int argc, char **argv) {
    long N = 256;                                   // multigrid.cpp:192
    int maxlvl = -1, shape = 1, nsmooth = 3, steps = -1, tower = MGX_TOWER_REFERENCE;
    double nu = -4 * 1e-4, tol = 1e-6;              // :235, :240
    bool cuda_file = false;
    int fp_mode = MGX_FP_BITWISE;
    std::string prefix;
    for (int a = 1; a < argc; ++a) {
        std::string k = argv[a];
        auto next = [&]() -> const char * {
            if (a + 1 >= argc) {
                fprintf(stderr, "missing value for %s\n", k.c_str());
                exit(2);
            }
            return argv[++a];
        };
        if (k == "-N") N = atol(next());
        else if (k == "-L") maxlvl = atoi(next());
        else if (k == "-nu") nu = atof(next());
        else if (k == "-steps") steps = atoi(next());
        else if (k == "-tol") tol = atof(next());
        else if (k == "-shape") shape = atoi(next());
        else if (k == "-nsmooth") nsmooth = atoi(next());
        else if (k == "-tower") tower = atoi(next());
        else if (k == "-out") prefix = next();
        else if (k == "-cuda") cuda_file = true;
        else if (k == "-fp") {
            const std::string v = next();
            if (v == "fma") fp_mode = MGX_FP_FMA;
            else if (v == "bitwise") fp_mode = MGX_FP_BITWISE;
            else {
                fprintf(stderr, "-fp takes bitwise or fma\n");
                return 2;
            }
        }
        else {
            fprintf(stderr, "unknown flag %s\n", k.c_str());
            return 2;
        }
    }
    if (maxlvl < 0) maxlvl = int(log2(N)) - 4;      // :193
    double dx = 1.0 / N;
    double dt = dx / 10;                            // :238
    double T = (steps < 0 ? 100 : steps) * dt;      // :239
    const size_t cnt = (size_t)(N + 1) * (N + 1);
    std::vector<double> u0(cnt), v1(cnt), v2(cnt), uTref(cnt), uTfast(cnt);
    die(mgx_init_problem(u0.data(), v1.data(), v2.data(), N, 0), "init_problem");

    auto t0 = std::chrono::steady_clock::now();
    timestepper(uTref.data(), u0.data(), v1.data(), v2.data(), nu, maxlvl, N, dt, T, tol, shape,
                nsmooth, tower);
    double s1 = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    // the reference's three stdout lines in its shapes (multigrid.cpp:246, :259,
    // :266: "<label> time, N = %i: %f s", "Error (...) = %10e"), with labels that
    // say what ran: leg 1 is the reference's op sequence through the gs.h-level
    // entry points, leg 2 the library's fused time stepper, both on one GPU.
    printf("\nGPU (reference op sequence, 1 MI355X) time, N = %i: %f s\n", (int)N, s1);

    mgx_options o;
    mgx_default_options(&o);
    o.shape = shape;
    o.nsmooth = nsmooth;
    o.tower_mode = tower;
    o.fp_mode = fp_mode;
    t0 = std::chrono::steady_clock::now();
    die(mgx_timestepper_ex(uTfast.data(), u0.data(), v1.data(), v2.data(), nu, maxlvl, N, dt, T,
                           dx, tol, &o, nullptr),
        "mgx_timestepper");
    double s2 = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("\nGPU (mgx_timestepper fused passes, 1 MI355X) time, N = %i: %f s\n", (int)N, s2);
    double error = 0;
    for (size_t p = 0; p < cnt; ++p) error += fabs(uTfast[p] - uTref[p]);
    printf("Error (compared to the referenced solution) = %10e\n", error);

    write_uT((prefix + "uT.txt").c_str(), uTref.data(), N);
    write_uT((prefix + "uTomp.txt").c_str(), uTfast.data(), N);
    if (cuda_file) write_uT((prefix + "uTcuda.txt").c_str(), uTfast.data(), N);
    return 0;
}
