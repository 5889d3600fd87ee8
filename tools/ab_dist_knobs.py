"""Per-rank level-0 cost on G virtual ranks under tuning knobs (interleaved).
    python tools/ab_dist_knobs.py key=v1,v2 [key=...] [--G 8] [--rounds 2]"""
import argparse, itertools, json, sys, time
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
from hpcclassmultigridproject_amd import _lib
ap = argparse.ArgumentParser()
ap.add_argument('knobs', nargs='*')
ap.add_argument('--G', type=int, default=8)
ap.add_argument('--N', type=int, default=16384)
ap.add_argument('--L', type=int, default=9)
ap.add_argument('--cycles', type=int, default=4)
ap.add_argument('--rounds', type=int, default=2)
a = ap.parse_args()
knobs = [(k, [int(x) for x in v.split(',')]) for k, v in (kv.split('=') for kv in a.knobs)]
N, L, G = a.N, a.L, a.G
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
mg = pkg.Multigrid(N, L, 1.0 / N / 10, -4e-4, device=0, local_parts=G)
mg.upload(u0, v1, v2); mg.rhs()
for rnd in range(a.rounds):
    for combo in itertools.product(*[v for _, v in knobs]):
        for (k, _), v in zip(knobs, combo):
            _lib.set_tuning(k, v)
        mg.run_cycles(1); mg.synchronize()
        mg.profile_reset(); mg.profile(True)
        t = time.perf_counter(); mg.run_cycles(a.cycles); mg.synchronize()
        ms = (time.perf_counter() - t) / a.cycles * 1e3
        lv = []
        for l in range(L):
            tl = 0.0
            for kind in _lib.KERNEL_NAMES:
                n, kms, _ = mg.profile_get(kind, l)
                tl += kms
            lv.append(round(tl / a.cycles / G, 4))
        mg.profile(False)
        key = ",".join(f"{k}={v}" for (k, _), v in zip(knobs, combo))
        print(rnd, key, json.dumps({"ms_per_rank": round(ms / G, 4), "per_level_per_rank": lv}),
              flush=True)
