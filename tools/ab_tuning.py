"""Interleaved A/B of tuning knobs in one process (MI355X_MICROARCH rule 24).
    python tools/ab_tuning.py key=v1,v2 [key2=...] [--rounds R] [--N 16384 --L 9]"""
import argparse, itertools, json, sys, time
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
from hpcclassmultigridproject_amd import _lib
ap = argparse.ArgumentParser()
ap.add_argument('knobs', nargs='+')
ap.add_argument('--rounds', type=int, default=3)
ap.add_argument('--cycles', type=int, default=5)
ap.add_argument('--N', type=int, default=16384)
ap.add_argument('--L', type=int, default=9)
a = ap.parse_args()
knobs = [(k, [int(x) for x in v.split(',')]) for k, v in (kv.split('=') for kv in a.knobs)]
N, L = a.N, a.L
dt = 1.0 / N / 10
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
mg = pkg.Multigrid(N, L, dt, -4e-4, device=0)
mg.upload(u0, v1, v2); mg.rhs()
res = {}
for rnd in range(a.rounds):
    for combo in itertools.product(*[v for _, v in knobs]):
        for (k, _), v in zip(knobs, combo):
            _lib.set_tuning(k, v)
        mg.run_cycles(1); mg.synchronize()
        mg.profile_reset(); mg.profile(True)
        t = time.perf_counter(); r = mg.run_cycles(a.cycles); mg.synchronize()
        ms = (time.perf_counter() - t) / a.cycles * 1e3
        d = {"ms": round(ms, 3)}
        for kind, name in _lib.KERNEL_NAMES.items():
            n, kms, _ = mg.profile_get(kind, 0)
            if n: d[name + "_L0"] = round(kms / n, 4)
        mg.profile(False)
        key = ",".join(f"{k}={v}" for (k, _), v in zip(knobs, combo))
        res.setdefault(key, []).append(d)
        print(rnd, key, json.dumps(d), flush=True)
print("SUMMARY")
for k, v in res.items():
    print(k, "median ms", sorted(x["ms"] for x in v)[len(v) // 2])
