import sys; sys.path.insert(0,'.')
import hpcclassmultigridproject_amd as pkg
N, L = 16384, 9
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
mg = pkg.Multigrid(N, L, 1.0/N/10, -4e-4, device=0)
mg.upload(u0, v1, v2); mg.rhs()
del u0, v1, v2
mg.run_cycles(1)
i0 = mg.coarse_iterations()
mg.run_cycles(10)
print("coarse iterations per cycle", (mg.coarse_iterations() - i0) / 10)
