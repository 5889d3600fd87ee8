"""Interleaved per-level A/B of tuning knobs in one process.
    python tools/ab_levels.py key=v1,v2 [key2=...] [--rounds R] [--N 16384 --L 9]
Per combination: wall ms per cycle (no events), then device ms per cycle of
every level (HIP events around every launch, all kernel kinds summed);
medians over the rounds at the end."""
import argparse, itertools, json, sys, time
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
from hpcclassmultigridproject_amd import _lib
ap = argparse.ArgumentParser()
ap.add_argument('knobs', nargs='*')
ap.add_argument('--rounds', type=int, default=3)
ap.add_argument('--cycles', type=int, default=5)
ap.add_argument('--N', type=int, default=16384)
ap.add_argument('--L', type=int, default=9)
ap.add_argument('--shape', type=int, default=1, help='1 V-cycle, 2 W-cycle')
ap.add_argument('--fp', choices=['bitwise', 'fma'], default='bitwise')
a = ap.parse_args()
knobs = [(k, [int(x) for x in v.split(',')]) for k, v in (kv.split('=') for kv in a.knobs)]
N, L = a.N, a.L
dt = 1.0 / N / 10
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
mg = pkg.Multigrid(N, L, dt, -4e-4, device=0, shape=a.shape,
                   fp_mode=_lib.FP_FMA if a.fp == 'fma' else _lib.FP_BITWISE)
mg.upload(u0, v1, v2); mg.rhs()
res = {}
for rnd in range(a.rounds):
    for combo in itertools.product(*[v for _, v in knobs]):
        for (k, _), v in zip(knobs, combo):
            _lib.set_tuning(k, v)
        mg.run_cycles(1); mg.synchronize()
        t = time.perf_counter(); mg.run_cycles(a.cycles); mg.synchronize()
        d = {"wall": (time.perf_counter() - t) / a.cycles * 1e3}
        mg.profile_reset(); mg.profile(True)
        mg.run_cycles(a.cycles); mg.synchronize()
        for lvl in range(L):
            d[f"L{lvl}"] = sum(mg.profile_get(kind, lvl)[1] for kind in _lib.KERNEL_NAMES) / a.cycles
        mg.profile(False)
        key = ",".join(f"{k}={v}" for (k, _), v in zip(knobs, combo)) or "default"
        res.setdefault(key, []).append(d)
        print(rnd, key, json.dumps({k: round(v, 4) for k, v in d.items()}), flush=True)
print("SUMMARY (medians, ms per cycle)")
for key, v in res.items():
    med = {f: sorted(x[f] for x in v)[len(v) // 2] for f in v[0]}
    print(key, json.dumps({k: round(x, 4) for k, x in med.items()}), flush=True)
