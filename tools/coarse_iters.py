"""Coarsest-level GS iterations per V-cycle at N=16384, L=9 (bench pattern)."""
import sys
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
N, L = 16384, 9
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
mg = pkg.Multigrid(N, L, 1.0 / N / 10, -4e-4, device=0)
mg.upload(u0, v1, v2)
mg.rhs()
for k in range(6):
    i0 = mg.coarse_iterations()
    r = mg.run_cycles(1)
    print(k, "coarse iterations", mg.coarse_iterations() - i0, "res", r, flush=True)
