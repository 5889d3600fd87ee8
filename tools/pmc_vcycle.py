"""Small driver for rocprofv3 --pmc passes: warm up, then a few V-cycles at N=16384.
    python tools/pmc_vcycle.py [N L cycles [fp_mode [generic]]]
fp_mode: fma (default, the bench's headline mode) or bitwise; generic = 1:
sep_velocity = zero_rows = 0 (the 2-D velocity path)."""
import sys
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
from hpcclassmultigridproject_amd import _lib
N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
L = int(sys.argv[2]) if len(sys.argv) > 2 else 9
cyc = int(sys.argv[3]) if len(sys.argv) > 3 else 3
fp = _lib.FP_BITWISE if len(sys.argv) > 4 and sys.argv[4] == "bitwise" else _lib.FP_FMA
if len(sys.argv) > 5 and sys.argv[5] == "1":
    _lib.set_tuning("sep_velocity", 0)
    _lib.set_tuning("zero_rows", 0)
dt = 1.0 / N / 10
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
mg = pkg.Multigrid(N, L, dt, -4e-4, device=0, fp_mode=fp)
mg.upload(u0, v1, v2)
del u0, v1, v2
mg.rhs()
mg.run_cycles(1)
print("res", mg.run_cycles(cyc), flush=True)
mg.close()
