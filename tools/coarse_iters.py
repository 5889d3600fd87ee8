"""Coarsest-level GS iterations per cycle at N=16384, L=9 (bench pattern).
    python tools/coarse_iters.py [--shape 1|2] [--fp bitwise|fma] [--cycles 6]
(per cycle: the iterations of all its coarsest solves; a W-cycle solves the
coarsest level 2^(L-1) times, 2 per launch)"""
import argparse
import sys
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
from hpcclassmultigridproject_amd import _lib
ap = argparse.ArgumentParser()
ap.add_argument('--shape', type=int, default=1)
ap.add_argument('--fp', choices=['bitwise', 'fma'], default='bitwise')
ap.add_argument('--cycles', type=int, default=6)
a = ap.parse_args()
N, L = 16384, 9
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
mg = pkg.Multigrid(N, L, 1.0 / N / 10, -4e-4, device=0, shape=a.shape,
                   fp_mode=_lib.FP_FMA if a.fp == 'fma' else _lib.FP_BITWISE)
mg.upload(u0, v1, v2)
mg.rhs()
solves = a.shape ** (L - 1)
for k in range(a.cycles):
    i0 = mg.coarse_iterations()
    r = mg.run_cycles(1)
    it = mg.coarse_iterations() - i0
    print(k, "coarse iterations", it, "per solve", round(it / solves, 2), "res", r, flush=True)
