"""A/B of the row-march kernels (tuning key march_kernel) in one process:
per-pass time of the finest-level passes and ms per V-cycle, interleaved.
    python tools/ab_march.py [--values 0,1,2] [--rounds 3]"""
import argparse, json, sys, time
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
from hpcclassmultigridproject_amd import _lib
ap = argparse.ArgumentParser()
ap.add_argument('--values', default='0,1,2')
ap.add_argument('--rounds', type=int, default=3)
ap.add_argument('--cycles', type=int, default=4)
ap.add_argument('--N', type=int, default=16384)
ap.add_argument('--L', type=int, default=9)
ap.add_argument('--fuse', default='3')
a = ap.parse_args()
N, L = a.N, a.L
dt = 1.0 / N / 10
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
mgs = {f: pkg.Multigrid(N, L, dt, -4e-4, device=0, fuse=int(f)) for f in a.fuse.split(',')}
for f, mg in mgs.items():
    mg.upload(u0, v1, v2); mg.rhs()
for rnd in range(a.rounds):
    for f, mg in mgs.items():
        for v in (int(x) for x in a.values.split(',')):
            _lib.set_tuning("march_kernel", v)
            mg.run_cycles(1); mg.synchronize()
            mg.profile_reset(); mg.profile(True, finest_only=True)
            t = time.perf_counter(); mg.run_cycles(a.cycles); mg.synchronize()
            ms = (time.perf_counter() - t) / a.cycles * 1e3
            d = {"fuse": f, "march_kernel": v, "ms_per_cycle": round(ms, 3)}
            for kind, name in _lib.KERNEL_NAMES.items():
                n, kms, b = mg.profile_get(kind, 0)
                if n:
                    d[name] = round(kms / n, 4)
            mg.profile(False)
            print(rnd, json.dumps(d), flush=True)
