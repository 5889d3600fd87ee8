"""The coarsest solve in isolation: N=64 with L=1 (mg_inner on the coarsest
level only) -- run under rocprofv3 --kernel-trace --stats to compare the
k_coarse_solve_lds duration with its duration inside a V-cycle."""
import sys
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
from hpcclassmultigridproject_amd import _lib
N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
L = int(sys.argv[2]) if len(sys.argv) > 2 else 1
u0, v1, v2 = pkg.init_problem(N, nthreads=4)
mg = pkg.Multigrid(N, L, 1.0 / 16384 / 10, -4e-4, device=0, fp_mode=_lib.FP_FMA)
mg.upload(u0, v1, v2)
mg.rhs()
for _ in range(200):
    mg.run_cycles(1)
mg.synchronize()
print("done", mg.coarse_iterations())
