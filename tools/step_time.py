"""Time steps at N=16384, interleaved over the values of one tuning key
(default step_fuse 0/1), and print one step's residual history.
    python tools/step_time.py [--N 16384 --L 9 --steps 3 --rounds 2
                               --key post_predict --values 0,100 --fp fma]"""
import argparse, sys, time
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
from hpcclassmultigridproject_amd import _lib
ap = argparse.ArgumentParser()
ap.add_argument('--N', type=int, default=16384)
ap.add_argument('--L', type=int, default=9)
ap.add_argument('--steps', type=int, default=3)
ap.add_argument('--rounds', type=int, default=2)
ap.add_argument('--key', default='step_fuse')
ap.add_argument('--values', default='0,1')
ap.add_argument('--fp', choices=['bitwise', 'fma'], default='bitwise')
a = ap.parse_args()
N, L = a.N, a.L
vals = [int(v) for v in a.values.split(',')]
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
mg = pkg.Multigrid(N, L, 1.0 / N / 10, -4e-4, device=0,
                   fp_mode=_lib.FP_FMA if a.fp == 'fma' else _lib.FP_BITWISE)
mg.upload(u0, v1, v2)
mg.rhs()
r0 = mg.residual_norm(0)
hist = [mg.run_cycles(1) / r0 for _ in range(5)]
print("residual / res0 after cycles 1..5:", " ".join(f"{h:.3e}" for h in hist), flush=True)
old = _lib.get_tuning(a.key)
ref = None
try:
    for rnd in range(a.rounds):
        for v in vals:
            _lib.set_tuning(a.key, v)
            mg.upload(u0, v1, v2)
            mg.synchronize()
            t = time.perf_counter()
            cyc = [mg.step(1e-6) for _ in range(a.steps)]
            mg.synchronize()
            ms = (time.perf_counter() - t) / a.steps * 1e3
            u = mg.download()
            same = ref is None or (u == ref).all()
            ref = u if ref is None else ref
            print(rnd, f"{a.key}={v}", f"{ms:.3f} ms/step", "cycles", cyc,
                  "bitwise" if same else "DIFFERS", flush=True)
finally:
    _lib.set_tuning(a.key, old)
