"""Small driver for rocprofv3 --pmc passes: warm up, then a few V-cycles at N=16384."""
import sys
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
L = int(sys.argv[2]) if len(sys.argv) > 2 else 9
cyc = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dt = 1.0 / N / 10
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
mg = pkg.Multigrid(N, L, dt, -4e-4, device=0)
mg.upload(u0, v1, v2)
del u0, v1, v2
mg.rhs()
mg.run_cycles(1)
print("res", mg.run_cycles(cyc), flush=True)
mg.close()
