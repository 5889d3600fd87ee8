"""Config 2 (N=4096, L=3, nu=2) timings: V-cycle, coarse iterations, timestep."""
import sys, time
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
from hpcclassmultigridproject_amd import _lib
N, L = 4096, 3
dt = 1.0 / N / 10
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
mg = pkg.Multigrid(N, L, dt, -4e-4, device=0, nsmooth=2)
mg.upload(u0, v1, v2); mg.rhs(); mg.run_cycles(1); mg.synchronize()
it0 = mg.coarse_iterations()
mg.profile_reset(); mg.profile(True)
t = time.perf_counter(); mg.run_cycles(10); mg.synchronize(); ms = (time.perf_counter() - t) / 10 * 1e3
print("ms per V-cycle", round(ms, 3), "coarse iters per cycle", (mg.coarse_iterations() - it0) / 10)
for kind, name in _lib.KERNEL_NAMES.items():
    n, kms, b = mg.profile_get(kind, -1)
    if n: print(" ", name, n / 10, "launches/cycle", round(kms / 10, 4), "ms/cycle")
mg.profile(False)
mg.upload(u0, v1, v2)
t = time.perf_counter(); cyc = [mg.step(1e-6) for _ in range(5)]; mg.synchronize()
print("ms per timestep", round((time.perf_counter() - t) / 5 * 1e3, 3), "cycles", cyc)
