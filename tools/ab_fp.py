"""Interleaved A/B of the arithmetic modes (mgx_options.fp_mode) in one process.
    python tools/ab_fp.py [--rounds R] [--cycles K] [--N 16384 --L 9] [--nsmooth 3]
Two contexts (bitwise, fma) on the same problem, alternated per round: wall ms
per cycle (no events), then device ms per cycle of every level (HIP events
around every launch) and of the cross pass; medians at the end, plus the
max |u_fma - u_bitwise| after the rounds."""
import argparse, json, sys, time
sys.path.insert(0, '.')
import numpy as np
import hpcclassmultigridproject_amd as pkg
from hpcclassmultigridproject_amd import _lib
ap = argparse.ArgumentParser()
ap.add_argument('--rounds', type=int, default=3)
ap.add_argument('--cycles', type=int, default=10)
ap.add_argument('--N', type=int, default=16384)
ap.add_argument('--L', type=int, default=9)
ap.add_argument('--nsmooth', type=int, default=3)
ap.add_argument('--generic', action='store_true', help='sep_velocity = zero_rows = 0')
a = ap.parse_args()
if a.generic:
    _lib.set_tuning("sep_velocity", 0)
    _lib.set_tuning("zero_rows", 0)
N, L = a.N, a.L
dt = 1.0 / N / 10
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
ctx = {}
for name, fp in (("bitwise", _lib.FP_BITWISE), ("fma", _lib.FP_FMA)):
    mg = pkg.Multigrid(N, L, dt, -4e-4, device=0, nsmooth=a.nsmooth, fp_mode=fp)
    mg.upload(u0, v1, v2)
    mg.rhs()
    ctx[name] = mg
del v1, v2
res = {}
for rnd in range(a.rounds):
    for name, mg in ctx.items():
        mg.run_cycles(1); mg.synchronize()
        t = time.perf_counter(); mg.run_cycles(a.cycles); mg.synchronize()
        d = {"wall": (time.perf_counter() - t) / a.cycles * 1e3}
        mg.profile_reset(); mg.profile(True)
        mg.run_cycles(a.cycles); mg.synchronize()
        for lvl in range(L):
            d[f"L{lvl}"] = sum(mg.profile_get(kind, lvl)[1] for kind in _lib.KERNEL_NAMES) / a.cycles
        d["xsmooth"] = mg.profile_get(_lib.K_XSMOOTH, 0)[1] / a.cycles
        mg.profile(False)
        res.setdefault(name, []).append(d)
        print(rnd, name, json.dumps({k: round(v, 4) for k, v in d.items()}), flush=True)
print("SUMMARY (medians, ms per cycle)")
for key, v in res.items():
    med = {f: sorted(x[f] for x in v)[len(v) // 2] for f in v[0]}
    print(key, json.dumps({k: round(x, 4) for k, x in med.items()}), flush=True)
ub = ctx["bitwise"].download(u0)
uf = ctx["fma"].download()
print("max|u_fma - u_bitwise| after", a.rounds * 3 * a.cycles + 2 * a.rounds, "cycles:",
      float(np.max(np.abs(uf - ub))), flush=True)
