"""Per-pass time of the finest-level fused smoothing pass vs sweeps per pass
(fuse = 1, 2, 3): equal HBM bytes per pass, compute growing with the sweeps.
Flat => HBM bound, proportional => compute/latency bound.
    python tools/ab_fuse.py [--N 16384 --L 9]"""
import argparse, json, sys, time
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
from hpcclassmultigridproject_amd import _lib
ap = argparse.ArgumentParser()
ap.add_argument('--N', type=int, default=16384)
ap.add_argument('--L', type=int, default=9)
ap.add_argument('--cycles', type=int, default=4)
a = ap.parse_args()
N, L = a.N, a.L
dt = 1.0 / N / 10
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
for fuse in (3, 2, 1, 3):
    mg = pkg.Multigrid(N, L, dt, -4e-4, device=0, fuse=fuse)
    mg.upload(u0, v1, v2); mg.rhs(); mg.run_cycles(1); mg.synchronize()
    mg.profile_reset(); mg.profile(True, finest_only=True)
    t = time.perf_counter(); mg.run_cycles(a.cycles); mg.synchronize()
    ms = (time.perf_counter() - t) / a.cycles * 1e3
    d = {"fuse": fuse, "ms_per_cycle": round(ms, 3)}
    for kind, name in _lib.KERNEL_NAMES.items():
        n, kms, b = mg.profile_get(kind, 0)
        if n:
            d[name] = {"launches": n, "ms_per_launch": round(kms / n, 4),
                       "GBs_algo": round(b / n / (kms / n * 1e-3) / 1e9)}
    mg.profile(False); mg.close()
    print(json.dumps(d), flush=True)
